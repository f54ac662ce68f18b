// Causal flash attention forward / backward for gfx950 (MI355X), bf16 in, fp32 accumulate (K6).
//
// Inputs are read straight out of the packed q|k|v GEMM output: element (b, t, head, d) of Q is at
// q[(b*T + t)*ld + head*HD + d] (same for K, V with their own base pointers); O / dO are
// [B*T, nh*HD] (row stride ldo).  GQA: query head h uses kv head h / (nh/nkv).
//
// MFMA: v_mfma_f32_32x32x16_bf16 (32x32 tile, K=16, 64-lane wave).  C/D layout on gfx950:
// col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5) for accumulator register r (0..15).
// A/B: lane l holds A[row l&31][k = 8*(l>>5) + j] and B[k = 8*(l>>5) + j][col l&31], j = 0..7.
// An accumulator X used as the next B operand (registers 8s..8s+7 -> k-step s) carries its rows in
// the permuted order 16s + 8(j>>2) + 4h + (j&3); the other operand is fetched in that same order
// with the transposing LDS read ds_read_b64_tr_b16 (4 consecutive rows of one column per lane).
//
// Three kernels, all with the same skeleton (4 waves x 32 rows on the lanes, 64-row tiles of the
// other operand streamed through LDS, register-staged prefetch of tile j+1 issued before the
// MFMAs of tile j and written to LDS after the next barrier):
//   fwd   per 128 queries: S^T = K Q^T (query on the lane -> online softmax is a register
//         reduction + one lane^32 exchange, the O rescale is lane-local), O^T += V^T P^T.
//   dq    per 128 queries: S^T, dP^T = V dO^T, dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T.
//   dkdv  per 128 keys (GQA: loops over the group's query heads): S = Q K^T, dP = dO V^T
//         (key on the lane), dV^T += dO^T P, dK^T += Q^T dS.
// No atomics and no cross-workgroup reduction anywhere: the backward is bitwise deterministic
// (DiLoCo replicas stay bit-identical), at the price of recomputing S/dP once more for dQ.
// LDS tiles are XOR-swizzled at 16-B granularity so the 32 lanes that read 32 different rows at
// one column spread over the banks; transposed reads compute the same swizzled addresses per lane.
// Causal: tiles past the diagonal are never loaded; fully masked (wave, tile) pairs are skipped;
// the longest query / key blocks are dispatched first.
#include "common.h"
#include <cstdlib>
#include <type_traits>

using namespace nd;

typedef __bf16 bfv8 __attribute__((ext_vector_type(8)));
typedef short sv4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0, 0);
}

__device__ __forceinline__ sv4 tr_read(const bf16_t* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((sv4 __attribute__((address_space(3)))*)(lds_ptr));
}

__device__ __forceinline__ bf16x8 cat4(sv4 a, sv4 b) {
  bf16x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

// Pack accumulator registers 8s..8s+7 into a bf16 MFMA operand fragment.
__device__ __forceinline__ bf16x8 pack_frag(const f32x16& x, int s) {
  u32x4 u;
  u[0] = pack2(x[8 * s + 0], x[8 * s + 1]);
  u[1] = pack2(x[8 * s + 2], x[8 * s + 3]);
  u[2] = pack2(x[8 * s + 4], x[8 * s + 5]);
  u[3] = pack2(x[8 * s + 6], x[8 * s + 7]);
  return __builtin_bit_cast(bf16x8, u);
}

__device__ __forceinline__ bf16x8 load16(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ bf16x8 zero8() { return bf16x8{0, 0, 0, 0, 0, 0, 0, 0}; }

// Element offset of (row, col) inside an XOR-swizzled [rows][HD] bf16 LDS tile (16-B chunks).
// The XOR key s(row) must keep BOTH access kinds conflict-free:
//  * row reads (ds_read_b128): 16 consecutive rows at one logical chunk -> 16 distinct bank slots;
//  * transposed reads (ds_read_b64_tr_b16): a 32-lane half reads rows r0..r0+3 (r0 % 4 == 0), 64 B
//    each, so rows that share a bank row must differ in the chunk bit that picks the 64-B half.
// HD=64 (two 128-B rows per 256-B bank row): s = bitreverse3((row >> 1) & 7)  [rows r0, r0+2 differ in bit 2]
// HD=128 (one row per bank row):             s = ((row & 3) << 2) | ((row >> 2) & 3)
// HD=32 (four 64-B rows per bank row):        s = (row >> 2) & 3
template <int HD>
__device__ __forceinline__ int soff(int row, int col) {
  int key;
  if constexpr (HD == 64) {
    const int u = (row >> 1) & 7;
    key = ((u & 1) << 2) | (u & 2) | ((u >> 2) & 1);
  } else if constexpr (HD == 128) {
    key = ((row & 3) << 2) | ((row >> 2) & 3);
  } else {
    key = (row >> 2) & 3;
  }
  const int ch = (col >> 3) ^ key;
  return row * HD + ch * 8 + (col & 7);
}

// A/B fragment with rows on the lanes: row `row`, k-step t, lane half h -> cols 16t + 8h .. +7
template <int HD>
__device__ __forceinline__ bf16x8 row_frag(const bf16_t* tile, int row, int t, int h) {
  return *reinterpret_cast<const bf16x8*>(&tile[soff<HD>(row, 16 * t + 8 * h)]);
}

// Transposed fragment for the permuted-k operand: rows r0 + 16s + 8(j>>2) + 4h + (j&3), column
// c0 + (lane & 31).  (g, i) = (lane >> 4, lane & 15).
template <int HD>
__device__ __forceinline__ bf16x8 tr_frag(const bf16_t* tile, int rbase, int cbase, int g, int i) {
  const int row = rbase + 4 * (g >> 1) + (i >> 2);
  const int col = cbase + 16 * (g & 1) + 4 * (i & 3);
  return cat4(tr_read(&tile[soff<HD>(row, col)]), tr_read(&tile[soff<HD>(row + 8, col)]));
}

// Rotate 8 (x1, x2) pairs held as two bf16x8 chunks: x1' = x1 c - x2 s, x2' = x2 c + x1 s
// (sgn = -1 applies the inverse rotation).  fp32 math, one rounding, same as nd_rope_inplace.
__device__ __forceinline__ void rope8(bf16x8& x1, bf16x8& x2, float4 c0, float4 c1, float4 s0, float4 s1, float sgn) {
  const float cc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  const float ss[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const float a0 = bf2f((bf16_t)x1[j]), a1 = bf2f((bf16_t)x1[j + 1]);
    const float b0 = bf2f((bf16_t)x2[j]), b1 = bf2f((bf16_t)x2[j + 1]);
    const float s0_ = sgn * ss[j], s1_ = sgn * ss[j + 1];
    const uint32_t u = pack2(a0 * cc[j] - b0 * s0_, a1 * cc[j + 1] - b1 * s1_);
    const uint32_t v = pack2(b0 * cc[j] + a0 * s0_, b1 * cc[j + 1] + a1 * s1_);
    x1[j] = (short)(u & 0xffff); x1[j + 1] = (short)(u >> 16);
    x2[j] = (short)(v & 0xffff); x2[j + 1] = (short)(v >> 16);
  }
}

// RoPE on register fragments f[t] = row[16t + 8h .. +7] (pairs t <-> t + NT/2, same lane).
template <int HD>
__device__ __forceinline__ void rope_frags(bf16x8* f, const float* cosT, const float* sinT, int pos, int h) {
  constexpr int NT = HD / 16;
#pragma unroll
  for (int t = 0; t < NT / 2; ++t) {
    const int d = 16 * t + 8 * h;
    const float4* cp = reinterpret_cast<const float4*>(cosT + (int64_t)pos * HD + d);
    const float4* sp = reinterpret_cast<const float4*>(sinT + (int64_t)pos * HD + d);
    rope8(f[t], f[t + NT / 2], cp[0], cp[1], sp[0], sp[1], 1.f);
  }
}

// Register-staged tile loader: ROWS x HD bf16 tile, 16-B chunks spread over 256 threads.
template <int ROWS, int HD>
struct Stage {
  static constexpr int CPR = HD / 8;
  static constexpr int N = (ROWS * CPR + 255) / 256;
  bf16x8 v[N];
  __device__ __forceinline__ void load(const bf16_t* base, int64_t stride, int row0, int nrows_valid) {
#pragma unroll
    for (int it = 0; it < N; ++it) {
      const int c = threadIdx.x + it * 256;
      const int row = c / CPR, ch = c % CPR;
      v[it] = zero8();
      if (c < ROWS * CPR && row0 + row < nrows_valid) v[it] = load16(base + (int64_t)(row0 + row) * stride + ch * 8);
    }
  }
  __device__ __forceinline__ void store(bf16_t* tile) const {
#pragma unroll
    for (int it = 0; it < N; ++it) {
      const int c = threadIdx.x + it * 256;
      if (c < ROWS * CPR) {
        const int row = c / CPR, ch = c % CPR;
        *reinterpret_cast<bf16x8*>(&tile[soff<HD>(row, ch * 8)]) = v[it];
      }
    }
  }
};

// Register-staged tile loader that applies RoPE (half-split rotation) on the fly: each thread owns
// a (chunk, chunk + HD/16) pair of one row, so both halves of every rotated pair are in its
// registers; cos/sin rows of the tile's positions come from the fp32 [T, HD] tables (L2-resident).
template <int ROWS, int HD>
struct StageRope {
  static constexpr int CPR = HD / 8, HP = CPR / 2;
  static constexpr int N = (ROWS * HP + 255) / 256;
  bf16x8 a[N], b[N];
  float4 c0[N], c1[N], s0[N], s1[N];
  __device__ __forceinline__ void load(const bf16_t* base, int64_t stride, int row0, int nrows_valid,
                                       const float* cosT, const float* sinT) {
#pragma unroll
    for (int it = 0; it < N; ++it) {
      const int p = threadIdx.x + it * 256;
      const int row = p / HP, ch = p % HP, pos = row0 + row;
      a[it] = zero8();
      b[it] = zero8();
      c0[it] = c1[it] = s0[it] = s1[it] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p < ROWS * HP && pos < nrows_valid) {
        a[it] = load16(base + (int64_t)pos * stride + ch * 8);
        b[it] = load16(base + (int64_t)pos * stride + (ch + HP) * 8);
        const float4* cp = reinterpret_cast<const float4*>(cosT + (int64_t)pos * HD + ch * 8);
        const float4* sp = reinterpret_cast<const float4*>(sinT + (int64_t)pos * HD + ch * 8);
        c0[it] = cp[0]; c1[it] = cp[1]; s0[it] = sp[0]; s1[it] = sp[1];
      }
    }
  }
  __device__ __forceinline__ void store(bf16_t* tile) const {
#pragma unroll
    for (int it = 0; it < N; ++it) {
      const int p = threadIdx.x + it * 256;
      if (p < ROWS * HP) {
        const int row = p / HP, ch = p % HP;
        bf16x8 ra = a[it], rb = b[it];
        rope8(ra, rb, c0[it], c1[it], s0[it], s1[it], 1.f);
        *reinterpret_cast<bf16x8*>(&tile[soff<HD>(row, ch * 8)]) = ra;
        *reinterpret_cast<bf16x8*>(&tile[soff<HD>(row, (ch + HP) * 8)]) = rb;
      }
    }
  }
};

template <bool ROPE, class S>
__device__ __forceinline__ void load_tile(S& st, const bf16_t* base, int64_t stride, int row0, int nvalid,
                                          const float* cosT, const float* sinT) {
  if constexpr (ROPE) st.load(base, stride, row0, nvalid, cosT, sinT);
  else st.load(base, stride, row0, nvalid);
}

constexpr float LOG2E = 1.4426950408889634f;

// x (op) x[lane ^ 32] with one v_permlane32_swap_b32 (gfx950) instead of __shfl_xor's LDS round
// trip (ds_bpermute + lgkmcnt wait).  With both operands = x the swap returns {x[lane & 31],
// x[32 + (lane & 31)]}: the pair's two values in the same order on both halves, so max and sum
// come out bitwise identical in lane l and l ^ 32.
__device__ __forceinline__ float pair_max32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair_sum32(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Raw v_exp_f32 (no denormal range fix-up: exp2f lowers to ~6 extra VALU ops per call).  Inputs
// here are <= 0 (scores minus a running max / LSE); results below 2^-126 flush to 0, harmless for P.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Softmax-arithmetic experiment switches, compiled into A/B side libraries only
// (`build.py --rev ... --extra-flags -DND_ATTN_X=<bits>`); the product library is built with 0.
//   1  s_setprio 1 around the S (/ dP) MFMA chains, the critical path of every kernel
//   2  packed f32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) for the score transform, the row sum and
//      the dS products -- bitwise the scalar forms (same per-element ops, same summation order)
//   4  forward: 4 of every 32 exp2s by round-to-nearest range reduction + a degree-6 polynomial on the
//      FMA pipe instead of v_exp_f32
//   8  s_setprio 1 around the P V (fwd) / dQ (dq) / dV dK (dkdv) MFMA chains
//  16  s_setprio 1 around the softmax / dS VALU block instead (the critical path between the two chains)
//  32  forward: 3 waves / SIMD (launch bound 3, 168 VGPRs, no spill) instead of 4
//  64  dK/dV: 64-query tiles at 3 waves / SIMD (launch bound 3: 33 KiB of LDS, <= 168 VGPRs) instead of
//      128-query tiles at 2
// 128  dK/dV (128-query tiles): the next tile's LDS-DMA pieces spread over the first three 32-query steps (Q, then
//      dO, then the row statistics) instead of all issued after the tile's barrier
// 256  forward: the two 32-key S chains interleaved MFMA by MFMA instead of one after the other
// 512  the round-5 wait placement (no settle() of the prologue fragment loads; A/B of the fix only)
#ifndef ND_ATTN_X
#define ND_ATTN_X 0
#endif
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v pk_fma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
template <int BIT>
__device__ __forceinline__ void xprio(int p) {
  if constexpr ((ND_ATTN_X & BIT) != 0) {
    if (p) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  }
}
// In-kernel segment stamps (diagnostic build only: -DND_ATTN_STAMP, never the product library; guide
// cdna_hip_programming.md §7 "In-kernel stamps"): s_memtime + lgkmcnt(0) as one statement between scheduling
// barriers; each segment's cycles are summed in scalar registers and every wave's lane 0 writes its sums to a
// buffer of its own (nd_attn_stamp_buffer) -- no output value depends on them.  Read SHARES, not run time.
#ifdef ND_ATTN_STAMP
__device__ unsigned long long* g_stamp_buf;
constexpr int kStampSeg = 10;
struct Stamps {
  unsigned long long last = 0, sum[kStampSeg] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  __device__ __forceinline__ static unsigned long long now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
  }
  __device__ __forceinline__ void start() { last = now(); }
  __device__ __forceinline__ void mark(int seg) {
    const unsigned long long t = now();
    sum[seg] += t - last;
    last = t;
  }
  __device__ __forceinline__ void flush(int kernel_id) {
    if ((threadIdx.x & 63) == 0 && g_stamp_buf) {
      const unsigned long long wid = (unsigned long long)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
      unsigned long long* o = g_stamp_buf + 1 + (wid * kStampSeg) + (unsigned long long)kernel_id * (1ull << 22);
      for (int k = 0; k < kStampSeg; ++k) o[k] = sum[k];
    }
  }
};
ND_API int nd_attn_stamp_buffer(void* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_buf), &p, sizeof(p));
}
#define ND_STAMP(x) x
#else
#define ND_STAMP(x)
#endif

// Retire the prologue's fragment loads (Q / dO in the forward and dQ kernels, K / V in dK/dV) BEFORE the tile
// loop.  Left alone, the compiler's wait-count pass keeps them "possibly outstanding" at the loop header (the
// loop body does not always use them: causally skipped tiles) and puts an s_waitcnt vmcnt(N) in front of their
// first use in EVERY iteration; the hardware counter also holds the LDS-DMA pieces the iteration has just issued
// (inline asm, invisible to the pass), so that wait stalled each tile / step until most of its prefetch had
// landed -- a full memory round trip per iteration.  An empty asm that consumes the registers makes the pass put
// one vmcnt(0) here instead.
template <int N>
__device__ __forceinline__ void settle(const bf16x8 (&f)[N]) {
  if constexpr ((ND_ATTN_X & 512) == 0) {
#pragma unroll
    for (int t = 0; t < N; ++t) asm volatile("" ::"v"(f[t]));
  }
}

// 2^x for x <= 0 without the transcendental unit: x = j + f, j = rint(x) by the 1.5 * 2^23 shifter,
// f in [-0.5, 0.5], 2^f by its degree-6 Taylor polynomial (relative error < 2e-7), 2^j into the exponent.
__device__ __forceinline__ float pexp2(float x) {
  const float xc = fmaxf(x, -126.f);
  const float t = xc + 12582912.f;
  const float f = xc - (t - 12582912.f);
  float p = fmaf(1.5403530e-4f, f, 1.3333558e-3f);
  p = fmaf(p, f, 9.6181291e-3f);
  p = fmaf(p, f, 5.5504109e-2f);
  p = fmaf(p, f, 2.4022651e-1f);
  p = fmaf(p, f, 6.9314718e-1f);
  p = fmaf(p, f, 1.f);
  const float r = __int_as_float(__float_as_int(p) + ((__float_as_int(t) - 0x4B400000) << 23));
  return x < -126.f ? 0.f : r;
}

// Store a [HD x 32] transposed accumulator (rows = head dim in registers, col = row index on the
// lane) as 8-B packed bf16 groups into row `out_row`.  With tables, the inverse RoPE rotation is
// applied first: head-dim rows d and d + HD/2 sit in the same lane (o <-> o + NO/2, or register
// r <-> r + 8 when HD = 32), so the un-rotation is lane-local.
template <int HD>
__device__ __forceinline__ void store_T(bf16_t* out_row, f32x16* acc, float mul, int h, const float* cosT,
                                        const float* sinT, int pos) {
  constexpr int NO = HD / 32;
  if (cosT) {
    const float* cr = cosT + (int64_t)pos * HD;
    const float* sr = sinT + (int64_t)pos * HD;
    if (NO >= 2) {
#pragma unroll
      for (int o = 0; o < NO / 2; ++o)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int d = o * 32 + 8 * g4 + 4 * h;
          const float4 c = *reinterpret_cast<const float4*>(cr + d);
          const float4 sn = *reinterpret_cast<const float4*>(sr + d);
          const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float y1 = acc[o][4 * g4 + q], y2 = acc[o + NO / 2][4 * g4 + q];
            acc[o][4 * g4 + q] = y1 * cc[q] + y2 * ss[q];
            acc[o + NO / 2][4 * g4 + q] = y2 * cc[q] - y1 * ss[q];
          }
        }
    } else {
#pragma unroll
      for (int g4 = 0; g4 < 2; ++g4) {
        const int d = 8 * g4 + 4 * h;
        const float4 c = *reinterpret_cast<const float4*>(cr + d);
        const float4 sn = *reinterpret_cast<const float4*>(sr + d);
        const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float y1 = acc[0][4 * g4 + q], y2 = acc[0][4 * g4 + 8 + q];
          acc[0][4 * g4 + q] = y1 * cc[q] + y2 * ss[q];
          acc[0][4 * g4 + 8 + q] = y2 * cc[q] - y1 * ss[q];
        }
      }
    }
  }
  // lanes l and l ^ 32 hold the two 4-wide halves of every 8-wide column group of one row: one
  // v_permlane32_swap per word gives lane half 0 the whole group 2p and half 1 the whole group 2p + 1,
  // so each lane writes 16-B chunks (NO x 2 stores) instead of 8-B ones (the epilogue store tail is
  // issue-bound)
#pragma unroll
  for (int o = 0; o < NO; ++o)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int ga = 2 * p, gb = 2 * p + 1;
      const uint32_t xa0 = pack2(acc[o][4 * ga + 0] * mul, acc[o][4 * ga + 1] * mul);
      const uint32_t xa1 = pack2(acc[o][4 * ga + 2] * mul, acc[o][4 * ga + 3] * mul);
      const uint32_t yb0 = pack2(acc[o][4 * gb + 0] * mul, acc[o][4 * gb + 1] * mul);
      const uint32_t yb1 = pack2(acc[o][4 * gb + 2] * mul, acc[o][4 * gb + 3] * mul);
      const auto s0 = __builtin_amdgcn_permlane32_swap(xa0, yb0, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(xa1, yb1, false, false);
      // half 0: {own group-ga words, partner's group-ga words}; half 1: {partner's gb, own gb}
      const int d = o * 32 + 8 * (h ? gb : ga);
      *reinterpret_cast<uint4*>(out_row + d) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
    }
}

namespace {
__device__ __forceinline__ void adma_b128(const void* sbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}
__device__ __forceinline__ void adma_b32(const void* sbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}
template <class T_>
__device__ __forceinline__ uint32_t lds_addr(const T_* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) T_*)p);
}
}  // namespace

// LDS-DMA of one ROWS x HD bf16 tile (row stride ld) into a soff<HD>-swizzled LDS tile by the 4 waves
// of a workgroup: 1-KiB wave-instructions of 64/CPR rows, per-lane source offsets fixed per kernel.
template <int HD, int ROWS, int NW = 4>  // NW waves share the tile
struct TileDma {
  static constexpr int CPR = HD / 8, RPI = 64 / CPR, IPW = (ROWS / RPI) / NW;
  uint32_t voff[IPW];
  int wu;
  __device__ __forceinline__ void init(int64_t ld) {
    const int lane = threadIdx.x & 63;
    wu = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const int row = (wu + NW * i) * RPI + lane / CPR, p = lane % CPR;
      const int lch = (soff<HD>(row, p * 8) - row * HD) / 8;  // XOR swizzle: physical p holds logical lch
      voff[i] = (uint32_t)(((int64_t)row * ld + lch * 8) * 2);
    }
  }
  // rows row0.. of `base` (already offset to the tile's first row) -> LDS tile at byte address `lds`
  __device__ __forceinline__ void issue(const bf16_t* base, uint32_t lds) const {
#pragma unroll
    for (int i = 0; i < IPW; ++i) adma_b128(base, voff[i], lds + (uint32_t)((wu + NW * i) * 1024));
  }
};

__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// =============================================================================== forward
// ABL (timing ablations only, wrong results; ND_ATTN_ABL): 1 no K/V DMA + no vmcnt wait, 2 no barrier,
// 4 no softmax (P = bf16(S)), 8 no P V MFMAs, 16 no S MFMAs (S = 0 + lane constant).  Bit 32 is a
// correct variant (cheaper mask, max tree, split row sum: needs T % 64 == 0), the default of the
// LDS-DMA path since the tile loop is unrolled (ND_ATTN_ABL=0 for the plain one).
// NW: waves per workgroup (4 or 8; 8 = 256-query blocks, every K/V tile DMA'd once per 256 queries: DMA only)
template <int HD, bool ROPE, bool DMA = false, bool PAD = false, int ABL = 0, int NW = 4>  // DMA: LDS-DMA K/V staging (!ROPE, T % 64 == 0)
__global__ void __launch_bounds__(64 * NW, (HD >= 128 ? 1 : (HD == 64 && DMA && !(ND_ATTN_X & 32)) ? 4 : 3)) attn_fwd_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                          const bf16_t* __restrict__ V, bf16_t* __restrict__ O,
                                                          float* __restrict__ LSE, int B, int nh, int nkv, int T,
                                                          int64_t ld, int64_t ldo, float scale,
                                                          const float* __restrict__ cosT, const float* __restrict__ sinT,
                                                          const int* __restrict__ KS, float thr, int order) {
  constexpr int BN = 64, NT = HD / 16, NO = HD / 32;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[2 * BN * HD];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[2 * BN * HD];

  constexpr int QB = 32 * NW;  // queries per workgroup
  static_assert(NW == 4 || (NW == 8 && DMA), "8-wave blocks: LDS-DMA staging only");
  const int nqb = (T + QB - 1) / QB, bh_count = B * nh;
  // order 0: q-block major (longest causal rows of every head first); 1: the q-blocks of one
  // (batch, head) run together on one XCD, so its K/V tiles are fetched from HBM once and re-read from L2
  int qb, bh;
  if (order) {
    // every q-block of every query head sharing one (batch, kv head) -- one K/V stream -- in one
    // contiguous id range, longest rows first inside it
    const int rep = nh / nkv, grp = nqb * rep;
    const int id = xcd_remap(blockIdx.x, nqb * bh_count);
    const int gi = id / grp, wi = id % grp;
    qb = nqb - 1 - wi / rep;
    bh = (gi / nkv) * nh + (gi % nkv) * rep + wi % rep;
  } else {
    qb = nqb - 1 - (int)(blockIdx.x / bh_count);  // longest causal rows first
    bh = blockIdx.x % bh_count;
  }
  const int b = bh / nh, head = bh % nh, kvh = head / (nh / nkv);
  const int ks = PAD ? KS[b] : 0;  // PAD (left-padded batch): keys < ks are masked for every query
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15;
  const int q0w = qb * QB + w * 32, qi = q0w + c32;
  const float c = scale * LOG2E;
  const bf16_t* Qb = Q + (int64_t)b * T * ld + (int64_t)head * HD;
  const bf16_t* Kb = K + (int64_t)b * T * ld + (int64_t)kvh * HD;
  const bf16_t* Vb = V + (int64_t)b * T * ld + (int64_t)kvh * HD;

  bf16x8 qf[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) qf[t] = qi < T ? load16(Qb + (int64_t)qi * ld + 16 * t + 8 * h) : zero8();
  if (ROPE && qi < T) rope_frags<HD>(qf, cosT, sinT, qi, h);
  settle(qf);
  f32x16 oacc[NO];
#pragma unroll
  for (int o = 0; o < NO; ++o) oacc[o] = f32x16{};
  float m = -INFINITY, l = 0.f;

  const int ntiles = (min(T, qb * QB + QB) + BN - 1) / BN;
  typename std::conditional<ROPE, StageRope<BN, HD>, Stage<BN, HD>>::type sk;
  Stage<BN, HD> sv;
  TileDma<HD, BN, NW> tdma;
  const uint32_t ks_a = lds_addr(Ks), vs_a = lds_addr(Vs);
  auto dma_issue = [&](int j) {
    const uint32_t off = (uint32_t)((j & 1) * BN * HD * 2);
    tdma.issue(Kb + (int64_t)j * BN * ld, ks_a + off);
    tdma.issue(Vb + (int64_t)j * BN * ld, vs_a + off);
  };
  ND_STAMP(Stamps stp; stp.start();)
  if constexpr (DMA) {
    // double-buffered tiles: wait(tile j) + barrier | DMA tile j+1 -> buf (j+1)&1 | compute(buf j&1)
    tdma.init(ld);
    dma_issue(0);
  } else {
    // double-buffered tiles: compute(buf j&1) | regs hold tile j+1 | store -> buf (j+1)&1 | ONE barrier
    load_tile<ROPE>(sk, Kb, ld, 0, T, cosT, sinT);
    sv.load(Vb, ld, 0, T);
    sk.store(Ks);
    sv.store(Vs);
    __syncthreads();
    if (ntiles > 1) {
      load_tile<ROPE>(sk, Kb, ld, BN, T, cosT, sinT);
      sv.load(Vb, ld, BN, T);
    }
  }
  // the tile loop is unrolled by the double-buffer parity (PAR = j & 1 at compile time): every LDS
  // fragment address is then a per-lane base plus an immediate offset, no per-tile address VALU
  auto tile = [&](int j, auto par_t) {
    int par_v;  // compile-time for the LDS-DMA loop, j & 1 for the register-staged one
    if constexpr (std::is_integral<decltype(par_t)>::value) par_v = par_t;
    else par_v = decltype(par_t)::value;
    const int PAR = par_v;
    const int k0 = j * BN;
    const bf16_t* Kt = Ks + PAR * (BN * HD);
    const bf16_t* Vt = Vs + PAR * (BN * HD);
    if constexpr (DMA) {
      ND_STAMP(stp.mark(7);)
      if constexpr (!(ABL & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ND_STAMP(stp.mark(0);)
      if constexpr (!(ABL & 2)) __syncthreads();
      ND_STAMP(stp.mark(1);)
      if constexpr (!(ABL & 1)) if (j + 1 < ntiles) dma_issue(j + 1);
      ND_STAMP(stp.mark(2);)
    }
    if (k0 <= q0w + 31) {  // else: whole tile above this wave's diagonal (wave-uniform)
      // K row fragments issued up front (V^T transposing reads stay next to their MFMAs: holding
      // them too costs the third wave per SIMD)
      bf16x8 ka[2][NT];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int t = 0; t < NT; ++t) ka[kt][t] = row_frag<HD>(Kt, kt * 32 + c32, t, h);
      f32x16 s[2];
      xprio<1>(1);
      if constexpr ((ND_ATTN_X & 256) != 0 && !(ABL & 16)) {
        // the two 32-key chains interleaved: two MFMAs between a K-fragment read and its use, not one
        s[0] = f32x16{};
        s[1] = f32x16{};
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) s[kt] = mfma32(ka[kt][t], qf[t], s[kt]);
      } else {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] = f32x16{};
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          if constexpr (ABL & 16) s[kt][t] += (float)ka[kt][t][0];
          else s[kt] = mfma32(ka[kt][t], qf[t], s[kt]);
        }
      }
      }
      xprio<1>(0);
      ND_STAMP(stp.mark(3);)
      if constexpr (ABL & 4) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int sidx = 0; sidx < 2; ++sidx) {
            const bf16x8 pf = pack_frag(s[kt], sidx);
#pragma unroll
            for (int o = 0; o < NO; ++o) {
              if constexpr (ABL & 8) oacc[o][sidx] += (float)pf[o];
              else oacc[o] = mfma32(tr_frag<HD>(Vt, kt * 32 + 16 * sidx, o * 32, g, i16), pf, oacc[o]);
            }
          }
        return;
      }
      xprio<16>(1);
      float mx;
      if constexpr (ABL & 32) {
        // variant 32: one compare + select per score against a per-lane limit (T % 64 == 0 here: no
        // key >= T), row max as four independent v_max3 chains
        if ((k0 + BN - 1 > q0w) || (PAD && k0 < ks)) {
          const int lim = qi - k0 - 4 * h, plim = ks - k0 - 4 * h;
#pragma unroll
          for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int ko = kt * 32 + (r & 3) + 8 * (r >> 2);
              if (ko > lim || (PAD && ko < plim)) s[kt][r] = -INFINITY;
            }
        }
        float a4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x16& x = s[i >> 1];
          const int r0 = (i & 1) * 8;
          a4[i] = max3f(x[r0], x[r0 + 1], x[r0 + 2]);
          a4[i] = max3f(a4[i], x[r0 + 3], x[r0 + 4]);
          a4[i] = max3f(a4[i], x[r0 + 5], x[r0 + 6]);
          a4[i] = max3f(a4[i], x[r0 + 7], a4[i]);
        }
        mx = pair_max32(max3f(a4[0], a4[1], max3f(a4[2], a4[3], a4[3]))) * c;
      } else {
        if ((k0 + BN - 1 > q0w) || (k0 + BN > T) || (PAD && k0 < ks)) {
#pragma unroll
          for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int key = k0 + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
              if (key > qi || key >= T || (PAD && key < ks)) s[kt][r] = -INFINITY;
            }
        }
        mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[kt][r]);
        mx = pair_max32(mx) * c;  // raw-score max -> log2 domain (c > 0)
      }
      // deferred max (guide T13): the running max moves only when the tile's max exceeds it by more
      // than thr (log2 units), so p <= 2^thr and the O rescale below is skipped on almost every tile.
      // Both lanes of a query pair see the same m / mx, so l and O get one consistent factor.
      const bool upd = mx > m + thr;
      const float mnew = upd ? mx : m;
      // a row with no visible key yet (a left-pad query: every key masked) keeps p = 0, l = 0
      const float mref = (PAD && mnew == -INFINITY) ? 0.f : mnew;
      const float alpha = upd ? fexp2(m - mref) : 1.f;
      m = mnew;
      float rs4[4] = {0.f, 0.f, 0.f, 0.f};  // variant 32: four independent partial sums
      float rs = 0.f;
      if constexpr ((ND_ATTN_X & 2) != 0 && (ABL & 32) != 0) {
        // packed: rsp[0] = (rs4[0], rs4[1]), rsp[1] = (rs4[2], rs4[3]) -- the scalar order exactly
        f2v rsp[2] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}};
        const f2v c2 = {c, c}, nm2 = {-mref, -mref};
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            f2v x = pk_fma(f2v{s[kt][r], s[kt][r + 1]}, c2, nm2);
            if constexpr ((ND_ATTN_X & 4) != 0) {
              x.x = fexp2(x.x);
              x.y = (r & 7) == 6 ? pexp2(x.y) : fexp2(x.y);
            } else {
              x.x = fexp2(x.x);
              x.y = fexp2(x.y);
            }
            s[kt][r] = x.x;
            s[kt][r + 1] = x.y;
            rsp[(r >> 1) & 1] += x;
          }
        rs = (rsp[0].x + rsp[0].y) + (rsp[1].x + rsp[1].y);
      } else {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float xx = fmaf(s[kt][r], c, -mref);
          const float p = ((ND_ATTN_X & 4) != 0 && (r & 7) == 7) ? pexp2(xx) : fexp2(xx);
          s[kt][r] = p;
          if constexpr (ABL & 32) rs4[r & 3] += p;
          else rs += p;
        }
      if constexpr (ABL & 32) rs = (rs4[0] + rs4[1]) + (rs4[2] + rs4[3]);
      }
      l = l * alpha + rs;
      if (__any(alpha != 1.f)) {
#pragma unroll
        for (int o = 0; o < NO; ++o) oacc[o] *= alpha;
      }
      xprio<16>(0);
      ND_STAMP(stp.mark(4);)
      xprio<8>(1);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int sidx = 0; sidx < 2; ++sidx) {
          const bf16x8 pf = pack_frag(s[kt], sidx);
#pragma unroll
          for (int o = 0; o < NO; ++o) {
            if constexpr (ABL & 8) oacc[o][sidx] += (float)pf[o];
            else oacc[o] = mfma32(tr_frag<HD>(Vt, kt * 32 + 16 * sidx, o * 32, g, i16), pf, oacc[o]);
          }
        }
      xprio<8>(0);
      ND_STAMP(stp.mark(5);)
    }
    if constexpr (!DMA) {
      if (j + 1 < ntiles) {
        sk.store(Ks + (PAR ^ 1) * (BN * HD));
        sv.store(Vs + (PAR ^ 1) * (BN * HD));
      }
      __syncthreads();
      if (j + 2 < ntiles) {
        load_tile<ROPE>(sk, Kb, ld, k0 + 2 * BN, T, cosT, sinT);
        sv.load(Vb, ld, k0 + 2 * BN, T);
      }
    }
    };
  if constexpr (DMA) {
    for (int j = 0; j < ntiles; j += 2) {
      tile(j, std::integral_constant<int, 0>{});
      if (j + 1 < ntiles) tile(j + 1, std::integral_constant<int, 1>{});
    }
  } else {
    for (int j = 0; j < ntiles; ++j) tile(j, j & 1);
  }
  ND_STAMP(stp.mark(7);)
  const float lt = pair_sum32(l);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (qi < T) {
    store_T<HD>(O + ((int64_t)b * T + qi) * ldo + (int64_t)head * HD, oacc, inv, h, nullptr, nullptr, 0);
    if (h == 0) LSE[((int64_t)b * nh + head) * T + qi] = m + log2f(lt);
  }
  ND_STAMP(stp.mark(6); stp.flush(0);)
}

// =============================================================================== backward
// delta[b, h, t] = sum_d dO * O   (fp32)
template <int HD>
__global__ void __launch_bounds__(256) attn_bwd_pre_kernel(const bf16_t* __restrict__ O, const bf16_t* __restrict__ dO,
                                                           float* __restrict__ delta, int B, int nh, int T, int64_t ldo) {
  constexpr int CPR = HD / 8;
  const int64_t rows = (int64_t)B * T * nh;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r = gid / CPR;
  const int ch = (int)(gid % CPR);
  float acc = 0.f;
  if (r < rows) {
    const int64_t bt = r / nh;
    const int head = (int)(r % nh);
    float a[8], d[8];
    Vec8<BF16>::load(O, bt * ldo + (int64_t)head * HD + ch * 8, a);
    Vec8<BF16>::load(dO, bt * ldo + (int64_t)head * HD + ch * 8, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += a[j] * d[j];
  }
#pragma unroll
  for (int off = CPR / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (r < rows && ch == 0) {
    const int64_t bt = r / nh;
    const int head = (int)(r % nh);
    const int64_t bb = bt / T, t = bt % T;
    delta[(bb * nh + head) * T + t] = acc;
  }
}

// dQ: per 128 queries of one (b, head), streaming 64-key K/V tiles up to the diagonal.
// PRE: the backward's row statistics are produced here instead of by attn_bwd_pre_kernel +
// attn_neg_stats_kernel: each lane already holds half of its query's dO row, so it loads the same
// half of O, dots, and one lane^32 exchange gives delta = rowsum(dO * O); the kernel then writes
// -delta and -LSE/c (the seeds of the dK/dV kernel, which therefore runs after this one).
// NW: waves per workgroup (8 = 256-query blocks, LDS-DMA only; see attn_fwd_kernel)
#ifndef ND_ATTN_DQ_OCC
#define ND_ATTN_DQ_OCC 2  // waves / SIMD the head_dim-64 dQ kernel is compiled for (A/B)
#endif
template <int HD, bool ROPE, bool ROPE_OUT, bool DMA = false, bool PRE = false, bool PAD = false, int NW = 4>  // DMA: LDS-DMA K/V staging
__global__ void __launch_bounds__(64 * NW, (HD >= 128 ? 1 : HD == 64 ? ND_ATTN_DQ_OCC : 2)) attn_bwd_dq_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                             const bf16_t* __restrict__ V, const bf16_t* __restrict__ dO,
                                                             const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                             bf16_t* __restrict__ dQ, int B, int nh, int nkv, int T,
                                                             int64_t ld, int64_t ldo, float scale,
                                                             const float* __restrict__ cosT, const float* __restrict__ sinT,
                                                             const bf16_t* __restrict__ O = nullptr,
                                                             float* __restrict__ NL = nullptr,
                                                             float* __restrict__ ND = nullptr,
                                                             const int* __restrict__ KS = nullptr, int order = 0) {
  constexpr int BN = 64, NT = HD / 16, NO = HD / 32;
  __shared__ __attribute__((aligned(16))) bf16_t Ks[2 * BN * HD];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[2 * BN * HD];

  constexpr int QB = 32 * NW;
  static_assert(NW == 4 || (NW == 8 && DMA), "8-wave blocks: LDS-DMA staging only");
  const int nqb = (T + QB - 1) / QB, bh_count = B * nh;
  int qb, bh;
  if (order) {  // see attn_fwd_kernel
    const int rep = nh / nkv, grp = nqb * rep;
    const int id = xcd_remap(blockIdx.x, nqb * bh_count);
    const int gi = id / grp, wi = id % grp;
    qb = nqb - 1 - wi / rep;
    bh = (gi / nkv) * nh + (gi % nkv) * rep + wi % rep;
  } else {
    qb = nqb - 1 - (int)(blockIdx.x / bh_count);
    bh = blockIdx.x % bh_count;
  }
  const int b = bh / nh, head = bh % nh, kvh = head / (nh / nkv);
  const int ks = PAD ? KS[b] : 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15;
  const int q0w = qb * QB + w * 32, qi = q0w + c32;
  const float c = scale * LOG2E;
  const bf16_t* Qb = Q + (int64_t)b * T * ld + (int64_t)head * HD;
  const bf16_t* dOb = dO + (int64_t)b * T * ldo + (int64_t)head * HD;
  const bf16_t* Kb = K + (int64_t)b * T * ld + (int64_t)kvh * HD;
  const bf16_t* Vb = V + (int64_t)b * T * ld + (int64_t)kvh * HD;

  ND_STAMP(Stamps stp; stp.start();)
  bf16x8 qf[NT], dof[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    qf[t] = qi < T ? load16(Qb + (int64_t)qi * ld + 16 * t + 8 * h) : zero8();
    dof[t] = qi < T ? load16(dOb + (int64_t)qi * ldo + 16 * t + 8 * h) : zero8();
  }
  if (ROPE && qi < T) rope_frags<HD>(qf, cosT, sinT, qi, h);
  const int64_t rowstat = ((int64_t)b * nh + head) * T;
  const float lse = qi < T ? LSE[rowstat + qi] : 0.f;
  float dlt;
  if constexpr (PRE) {
    float acc = 0.f;
    if (qi < T) {
      const bf16_t* Orow = O + ((int64_t)b * T + qi) * ldo + (int64_t)head * HD;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const bf16x8 of = load16(Orow + 16 * t + 8 * h);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc = fmaf(bf2f((bf16_t)of[j]), bf2f((bf16_t)dof[t][j]), acc);
      }
    }
    dlt = pair_sum32(acc);
    if (qi < T && h == 0) {
      ND[rowstat + qi] = -dlt;
      NL[rowstat + qi] = -lse * (1.f / c);
    }
  } else {
    dlt = qi < T ? DELTA[rowstat + qi] : 0.f;
  }
  settle(qf);
  settle(dof);
  f32x16 dq[NO];
#pragma unroll
  for (int o = 0; o < NO; ++o) dq[o] = f32x16{};

  const int ntiles = (min(T, qb * QB + QB) + BN - 1) / BN;
  typename std::conditional<ROPE, StageRope<BN, HD>, Stage<BN, HD>>::type sk;
  Stage<BN, HD> sv;
  TileDma<HD, BN, NW> tdma;
  const uint32_t ks_a = lds_addr(Ks), vs_a = lds_addr(Vs);
  auto dma_issue = [&](int j) {
    const uint32_t off = (uint32_t)((j & 1) * BN * HD * 2);
    tdma.issue(Kb + (int64_t)j * BN * ld, ks_a + off);
    tdma.issue(Vb + (int64_t)j * BN * ld, vs_a + off);
  };
  if constexpr (DMA) {
    tdma.init(ld);
    dma_issue(0);
  } else {
    load_tile<ROPE>(sk, Kb, ld, 0, T, cosT, sinT);
    sv.load(Vb, ld, 0, T);
    sk.store(Ks);
    sv.store(Vs);
    __syncthreads();
    if (ntiles > 1) {
      load_tile<ROPE>(sk, Kb, ld, BN, T, cosT, sinT);
      sv.load(Vb, ld, BN, T);
    }
  }
  ND_STAMP(stp.mark(9);)
  for (int j = 0; j < ntiles; ++j) {
    const int k0 = j * BN;
    const bf16_t* Kt = Ks + (j & 1) * (BN * HD);
    const bf16_t* Vt = Vs + (j & 1) * (BN * HD);
    if constexpr (DMA) {
      ND_STAMP(stp.mark(7);)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ND_STAMP(stp.mark(0);)
      __syncthreads();
      ND_STAMP(stp.mark(1);)
      if (j + 1 < ntiles) dma_issue(j + 1);
      ND_STAMP(stp.mark(2);)
    }
    if (k0 <= q0w + 31) {
      const bool diag = (k0 + BN - 1 > q0w) || (k0 + BN > T) || (qi >= T) || (PAD && k0 < ks);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        if (k0 + kt * 32 > q0w + 31) continue;  // this 32-key half is above the wave's diagonal
        ND_STAMP(stp.mark(7);)
        // fragments issued up front (row reads for S^T / dP^T, transposing reads for dQ)
        bf16x8 ka[NT], va[NT], tk[2][NO];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          ka[t] = row_frag<HD>(Kt, kt * 32 + c32, t, h);
          va[t] = row_frag<HD>(Vt, kt * 32 + c32, t, h);
        }
#pragma unroll
        for (int sidx = 0; sidx < 2; ++sidx)
#pragma unroll
          for (int o = 0; o < NO; ++o) tk[sidx][o] = tr_frag<HD>(Kt, kt * 32 + 16 * sidx, o * 32, g, i16);
        ND_STAMP(stp.mark(3);)
        f32x16 s = f32x16{}, dp = f32x16{};
        xprio<1>(1);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          s = mfma32(ka[t], qf[t], s);
          dp = mfma32(va[t], dof[t], dp);
        }
        xprio<1>(0);
        ND_STAMP(stp.mark(4);)
        xprio<16>(1);
        if (!diag) {
          if constexpr ((ND_ATTN_X & 2) != 0) {
            const f2v c2 = {c, c}, nl2 = {-lse, -lse}, nd2 = {-dlt, -dlt};
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              f2v x = pk_fma(f2v{s[r], s[r + 1]}, c2, nl2);
              x.x = fexp2(x.x);
              x.y = fexp2(x.y);
              const f2v y = x * (f2v{dp[r], dp[r + 1]} + nd2);
              dp[r] = y.x;
              dp[r + 1] = y.y;
            }
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) dp[r] = fexp2(fmaf(s[r], c, -lse)) * (dp[r] - dlt);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            const float p = (key <= qi && key < T && qi < T && (!PAD || key >= ks)) ? fexp2(fmaf(s[r], c, -lse)) : 0.f;
            dp[r] = p * (dp[r] - dlt);
          }
        }
        xprio<16>(0);
        ND_STAMP(stp.mark(5);)
        xprio<8>(1);
#pragma unroll
        for (int sidx = 0; sidx < 2; ++sidx) {
          const bf16x8 dsf = pack_frag(dp, sidx);
#pragma unroll
          for (int o = 0; o < NO; ++o) dq[o] = mfma32(tk[sidx][o], dsf, dq[o]);
        }
        xprio<8>(0);
        ND_STAMP(stp.mark(6);)
      }
    }
    if constexpr (!DMA) {
      if (j + 1 < ntiles) {
        sk.store(Ks + ((j + 1) & 1) * (BN * HD));
        sv.store(Vs + ((j + 1) & 1) * (BN * HD));
      }
      __syncthreads();
      if (j + 2 < ntiles) {
        load_tile<ROPE>(sk, Kb, ld, k0 + 2 * BN, T, cosT, sinT);
        sv.load(Vb, ld, k0 + 2 * BN, T);
      }
    }
  }
  ND_STAMP(stp.mark(7);)
  if (qi < T)
    store_T<HD>(dQ + ((int64_t)b * T + qi) * ld + (int64_t)head * HD, dq, scale, h, ROPE_OUT ? cosT : nullptr, sinT, qi);
  ND_STAMP(stp.mark(8); if (PRE && DMA) stp.flush(2);)
}

// dK, dV: per 128 keys of one (b, kv head); loops over the GQA group's query heads and 64-query
// tiles from the diagonal to T.
template <int HD, bool ROPE, bool ROPE_OUT, bool PAD = false>
__global__ void __launch_bounds__(256, (HD >= 128 ? 1 : 2)) attn_bwd_dkdv_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                               const bf16_t* __restrict__ V, const bf16_t* __restrict__ dO,
                                                               const float* __restrict__ LSE,
                                                               const float* __restrict__ DELTA, bf16_t* __restrict__ dK,
                                                               bf16_t* __restrict__ dV, int B, int nh, int nkv, int T,
                                                               int64_t ld, int64_t ldo, float scale,
                                                               const float* __restrict__ cosT,
                                                               const float* __restrict__ sinT,
                                                               const int* __restrict__ KS, int order) {
  constexpr int BQ = 64, NT = HD / 16, NO = HD / 32;
  __shared__ __attribute__((aligned(16))) bf16_t Qs[2 * BQ * HD];
  __shared__ __attribute__((aligned(16))) bf16_t dOs[2 * BQ * HD];
  __shared__ __attribute__((aligned(16))) float lse_s[2 * BQ];
  __shared__ __attribute__((aligned(16))) float del_s[2 * BQ];

  const int nkb = (T + 127) / 128, bk_count = B * nkv, rep = nh / nkv;
  int kb, bk;  // order 1: the key blocks of one (batch, kv head) together on one XCD (Q / dO from L2)
  if (order & 1) {
    const int id = xcd_remap(blockIdx.x, nkb * bk_count);
    bk = id / nkb;
    kb = id % nkb;
  } else {
    kb = (int)(blockIdx.x / bk_count);  // small kb = longest query range: dispatched first
    bk = blockIdx.x % bk_count;
  }
  const int b = bk / nkv, kvh = bk % nkv;
  const int ks = PAD ? KS[b] : 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15;
  const int kw0 = kb * 128 + w * 32, key = kw0 + c32;
  const float c = scale * LOG2E;
  const bf16_t* Kb = K + (int64_t)b * T * ld + (int64_t)kvh * HD;
  const bf16_t* Vb = V + (int64_t)b * T * ld + (int64_t)kvh * HD;
  (void)nkb;

  bf16x8 kf[NT], vf[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    kf[t] = key < T ? load16(Kb + (int64_t)key * ld + 16 * t + 8 * h) : zero8();
    vf[t] = key < T ? load16(Vb + (int64_t)key * ld + 16 * t + 8 * h) : zero8();
  }
  if (ROPE && key < T) rope_frags<HD>(kf, cosT, sinT, key, h);
  settle(kf);
  settle(vf);
  f32x16 dk[NO], dv[NO];
#pragma unroll
  for (int o = 0; o < NO; ++o) { dk[o] = f32x16{}; dv[o] = f32x16{}; }

  const int qstart = (kb * 128) / BQ * BQ;
  const int ntq = (T - qstart + BQ - 1) / BQ;
  const int nit = ntq * rep;
  typename std::conditional<ROPE, StageRope<BQ, HD>, Stage<BQ, HD>>::type sq;
  Stage<BQ, HD> sd;
  float lse_n = 0.f, del_n = 0.f;
  auto prefetch = [&](int it) {
    const int head = kvh * rep + it / ntq;
    const int q0 = qstart + (it % ntq) * BQ;
    load_tile<ROPE>(sq, Q + (int64_t)b * T * ld + (int64_t)head * HD, ld, q0, T, cosT, sinT);
    sd.load(dO + (int64_t)b * T * ldo + (int64_t)head * HD, ldo, q0, T);
    if (threadIdx.x < BQ) {  // stored negated: they seed the S / dP accumulators
      const int qq = q0 + threadIdx.x;
      const int64_t rs = ((int64_t)b * nh + head) * T;
      lse_n = qq < T ? -LSE[rs + qq] / c : 0.f;
      del_n = qq < T ? -DELTA[rs + qq] : 0.f;
    }
  };
  auto commit = [&](int buf) {
    sq.store(Qs + buf * (BQ * HD));
    sd.store(dOs + buf * (BQ * HD));
    if (threadIdx.x < BQ) {
      lse_s[buf * BQ + threadIdx.x] = lse_n;
      del_s[buf * BQ + threadIdx.x] = del_n;
    }
  };
  prefetch(0);
  commit(0);
  __syncthreads();
  if (nit > 1) prefetch(1);
  for (int it = 0; it < nit; ++it) {
    const int q0 = qstart + (it % ntq) * BQ;
    const int buf = it & 1;
    const bf16_t* Qt = Qs + buf * (BQ * HD);
    const bf16_t* dOt = dOs + buf * (BQ * HD);
    const float* lt = lse_s + buf * BQ;
    const float* dt = del_s + buf * BQ;
#pragma unroll
    for (int qs = 0; qs < BQ / 32; ++qs) {
      const int qsub = q0 + qs * 32;
      if (kw0 > qsub + 31 || kw0 >= T) continue;  // wave-uniform: no query >= any of our keys
      // All LDS fragments of this step are issued up front (row reads for S / dP, transposing reads
      // for dV / dK) so their latency hides behind the MFMA chains and the softmax VALU instead of
      // being exposed one s_waitcnt at a time.
      bf16x8 qa[NT], da[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        qa[t] = row_frag<HD>(Qt, qs * 32 + c32, t, h);
        da[t] = row_frag<HD>(dOt, qs * 32 + c32, t, h);
      }
      f32x16 s, dp;  // seeded with -LSE / c and -delta of each query row
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int qr = qs * 32 + 8 * r4 + 4 * h;
        const float4 l4 = *reinterpret_cast<const float4*>(lt + qr);
        const float4 d4 = *reinterpret_cast<const float4*>(dt + qr);
        s[4 * r4 + 0] = l4.x; s[4 * r4 + 1] = l4.y; s[4 * r4 + 2] = l4.z; s[4 * r4 + 3] = l4.w;
        dp[4 * r4 + 0] = d4.x; dp[4 * r4 + 1] = d4.y; dp[4 * r4 + 2] = d4.z; dp[4 * r4 + 3] = d4.w;
      }
      bf16x8 tdo[2][NO], tq[2][NO];
#pragma unroll
      for (int sidx = 0; sidx < 2; ++sidx)
#pragma unroll
        for (int o = 0; o < NO; ++o) {
          tdo[sidx][o] = tr_frag<HD>(dOt, qs * 32 + 16 * sidx, o * 32, g, i16);
          tq[sidx][o] = tr_frag<HD>(Qt, qs * 32 + 16 * sidx, o * 32, g, i16);
        }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        s = mfma32(qa[t], kf[t], s);
        dp = mfma32(da[t], vf[t], dp);
      }
      const bool diag = (kw0 + 31 > qsub) || (qsub + 31 >= T) || (key >= T) || (PAD && kw0 < ks);
      if (!diag) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(s[r] * c);
          s[r] = p;
          dp[r] = p * dp[r];
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qq = qsub + (r & 3) + 8 * (r >> 2) + 4 * h;
          const float p = (key <= qq && qq < T && key < T && (!PAD || key >= ks)) ? fexp2(s[r] * c) : 0.f;
          s[r] = p;
          dp[r] = p * dp[r];
        }
      }
#pragma unroll
      for (int sidx = 0; sidx < 2; ++sidx) {
        const bf16x8 pf = pack_frag(s, sidx);
        const bf16x8 dsf = pack_frag(dp, sidx);
#pragma unroll
        for (int o = 0; o < NO; ++o) {
          dv[o] = mfma32(tdo[sidx][o], pf, dv[o]);
          dk[o] = mfma32(tq[sidx][o], dsf, dk[o]);
        }
      }
    }
    if (it + 1 < nit) commit((it + 1) & 1);
    __syncthreads();
    if (it + 2 < nit) prefetch(it + 2);
  }
  if (key < T) {
    store_T<HD>(dK + ((int64_t)b * T + key) * ld + (int64_t)kvh * HD, dk, scale, h, ROPE_OUT ? cosT : nullptr, sinT, key);
    store_T<HD>(dV + ((int64_t)b * T + key) * ld + (int64_t)kvh * HD, dv, 1.f, h, nullptr, nullptr, 0);
  }
}

// ------------------------------------------------------------------------------------ launchers
// Launch-time switches, read ONCE when the library loads (never per launch).  Only correct variants are
// selectable in the product library; the wrong-result timing ablations (ABL bits other than the
// forward's 32) are compiled only into a -DND_ABLATION build (`python -m nanodiloco_amd.csrc.build
// --ablation` -> _lib/alt/libnd_kernels_ablation.so), so a stray ND_ATTN_*ABL variable cannot change
// what a training job computes.
#ifndef ND_ATTN_DKDV_ORDER_DEFAULT
#define ND_ATTN_DKDV_ORDER_DEFAULT 0
#endif
struct AttnEnv {
  int order = 1;        // ND_ATTN_ORDER: grid order (see attn_fwd_kernel)
  int dkdv_order = ND_ATTN_DKDV_ORDER_DEFAULT;   // ND_ATTN_DKDV_ORDER: bit 0 group the key blocks of one (batch, kv head), bit 1 descending query walk
  float thr = 8.f;      // ND_ATTN_THR: deferred-max threshold (log2 units; 0 = move the max on every increase)
  bool fwd_reg = false; // ND_ATTN_FWD=r: register-staged forward
  int fwd_var = 32;     // ND_ATTN_ABL: 32 (cheaper mask / v_max3 tree, 1.007-1.024x) or 0 (plain)
  bool fwd_w8 = false, dq_w8 = false, dkdv_w8 = false;  // ND_ATTN_{FWD,DQ,DKDV}_W=8: 256-row blocks
  int dkdv_nb = 0;      // ND_ATTN_DKDV_NB=2..4: 64-query dK/dV tiles with NB LDS buffers
  bool dkdv_reg = false;   // ND_ATTN_DKDV=r: register-staged dK/dV (unfused backward)
  bool dkdv_bq64 = false;  // ND_DKDV_BQ=64: 64-query tiles (unfused backward)
  int fwd_abl = 0, dkdv_abl = 0;  // ND_ATTN_ABL / ND_ATTN_DKDV_ABL timing ablations: ND_ABLATION builds only
};
static const AttnEnv g_attn = [] {
  AttnEnv c;
  auto s = [](const char* k) { return getenv(k); };
  if (const char* e = s("ND_ATTN_ORDER")) c.order = atoi(e);
  if (const char* e = s("ND_ATTN_DKDV_ORDER")) c.dkdv_order = atoi(e);
  if (const char* e = s("ND_ATTN_THR")) c.thr = (float)atof(e);
  if (const char* e = s("ND_ATTN_FWD")) c.fwd_reg = e[0] == 'r';
  if (const char* e = s("ND_ATTN_ABL")) {
    const int v = atoi(e);
    if (v == 0 || v == 32) c.fwd_var = v;
#ifdef ND_ABLATION
    else c.fwd_abl = v;
#endif
  }
  if (const char* e = s("ND_ATTN_FWD_W")) c.fwd_w8 = e[0] == '8';
  if (const char* e = s("ND_ATTN_DQ_W")) c.dq_w8 = e[0] == '8';
  if (const char* e = s("ND_ATTN_DKDV_W")) c.dkdv_w8 = e[0] == '8';
  if (const char* e = s("ND_ATTN_DKDV_NB"); e && e[0] >= '2' && e[0] <= '4') c.dkdv_nb = e[0] - '0';
  if (const char* e = s("ND_ATTN_DKDV")) c.dkdv_reg = e[0] == 'r';
  if (const char* e = s("ND_DKDV_BQ")) c.dkdv_bq64 = e[0] == '6';
#ifdef ND_ABLATION
  if (const char* e = s("ND_ATTN_DKDV_ABL")) c.dkdv_abl = atoi(e);
#endif
  return c;
}();
static int attn_order() { return g_attn.order; }
// bit 0: a (batch, head)'s key blocks consecutive on one XCD (MHA only); bit 1: descending query walk
// (LDS-DMA dK/dV kernel)
static int dkdv_order(int nh, int nkv) { return ((g_attn.dkdv_order & 1) && nh == nkv ? 1 : 0) | (g_attn.dkdv_order & 2); }

// wrong-result ablation builds only (timing): ABL bits of attn_fwd_kernel / attn_bwd_dkdv_dma_kernel
#ifdef ND_ABLATION
ND_API int nd_attn_ablation_build() { return 1; }
#endif

template <int HD, bool PAD>
static int fwd_launch(const void* q, const void* k, const void* v, void* o, float* lse, int B, int nh, int nkv, int T,
                      int64_t ld, int64_t ldo, const float* cosT, const float* sinT, float scale, const int* ks,
                      hipStream_t s) {
  const int nqb = (T + 127) / 128;
  const dim3 g(nqb * B * nh), b(256);
  // deferred-max threshold (log2 units; ND_ATTN_THR for A/B, 0 = move the max on every increase)
  const float thr = g_attn.thr;
  if (cosT)
    hipLaunchKernelGGL((attn_fwd_kernel<HD, true, false, PAD>), g, b, 0, s, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                       (bf16_t*)o, lse, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, ks, thr, attn_order());
  else if (T % 64 == 0 && !g_attn.fwd_reg) {
#define ND_ABL(A)                                                                                                  \
  case A:                                                                                                          \
    hipLaunchKernelGGL((attn_fwd_kernel<HD, false, true, PAD, A>), g, b, 0, s, (const bf16_t*)q, (const bf16_t*)k, \
                       (const bf16_t*)v, (bf16_t*)o, lse, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, ks, thr,      \
                       attn_order());                                                                              \
    break;
#define ND_ABL8(A)                                                                                                   \
  case A:                                                                                                            \
    hipLaunchKernelGGL((attn_fwd_kernel<HD, false, true, PAD, A, 8>), g8, b8, 0, s, (const bf16_t*)q, (const bf16_t*)k, \
                       (const bf16_t*)v, (bf16_t*)o, lse, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, ks, thr,        \
                       attn_order());                                                                                \
    break;
    const int abl = PAD ? 0 : (g_attn.fwd_abl ? g_attn.fwd_abl : g_attn.fwd_var);
    bool w8 = false;
    if constexpr (HD >= 64) w8 = g_attn.fwd_w8;  // HD 32: a 64-row tile is 4 DMA pieces, < 8 waves
    if (w8) {
      const dim3 g8((T + 255) / 256 * B * nh), b8(512);
      switch (abl) {
#ifdef ND_ABLATION
        ND_ABL8(1) ND_ABL8(3) ND_ABL8(4) ND_ABL8(28)
#endif
        ND_ABL8(32)
        default: ND_ABL8(0)
      }
    } else {
      switch (abl) {
#ifdef ND_ABLATION
        ND_ABL(1) ND_ABL(2) ND_ABL(3) ND_ABL(4) ND_ABL(7) ND_ABL(8) ND_ABL(12) ND_ABL(16) ND_ABL(20) ND_ABL(24) ND_ABL(28)
#endif
        ND_ABL(32)
        default: ND_ABL(0)
      }
    }
#undef ND_ABL8
#undef ND_ABL
  }
  else
    hipLaunchKernelGGL((attn_fwd_kernel<HD, false, false, PAD>), g, b, 0, s, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v,
                       (bf16_t*)o, lse, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, ks, thr, attn_order());
  ND_LAUNCH_CHECK();
}

// cosT/sinT: fp32 [T, hd] RoPE tables (nullptr = q/k already rotated).  q/k/v are then the RAW
// projection outputs and the kernel rotates q and k on load.
// ks: per-sequence key start [B] (int32, device; nullptr = none) for left-padded batches: query q
// attends to keys ks[b] <= k <= q -- HF's causal & padding mask.  A pad query (q < ks[b]) sees no key
// and outputs 0 (what torch SDPA returns for a fully masked row, i.e. the reference's HF model).
ND_API int nd_attn_fwd_ks(const void* q, const void* k, const void* v, void* o, float* lse, int B, int nh, int nkv,
                          int T, int hd, int64_t ld, int64_t ldo, const float* cosT, const float* sinT, float scale,
                          const int* ks, hipStream_t s) {
  if (nh % nkv || (ld % 8) || (ldo % 8)) return (int)hipErrorInvalidValue;
  switch (hd) {
#define ND_FW(H) \
    case H: return ks ? fwd_launch<H, true>(q, k, v, o, lse, B, nh, nkv, T, ld, ldo, cosT, sinT, scale, ks, s) \
                      : fwd_launch<H, false>(q, k, v, o, lse, B, nh, nkv, T, ld, ldo, cosT, sinT, scale, ks, s);
    ND_FW(32)
    ND_FW(64)
    ND_FW(128)
#undef ND_FW
    default: return (int)hipErrorInvalidValue;
  }
}

ND_API int nd_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int nh, int nkv, int T,
                       int hd, int64_t ld, int64_t ldo, const float* cosT, const float* sinT, float scale,
                       hipStream_t s) {
  return nd_attn_fwd_ks(q, k, v, o, lse, B, nh, nkv, T, hd, ld, ldo, cosT, sinT, scale, nullptr, s);
}

ND_API int nd_attn_bwd_pre(const void* o, const void* dout, float* delta, int B, int nh, int T, int64_t hd,
                           int64_t ldo, hipStream_t s) {
  const int64_t threads = (int64_t)B * T * nh * (hd / 8);
  const unsigned grid = (unsigned)((threads + 255) / 256);
  switch (hd) {
    case 32: hipLaunchKernelGGL(attn_bwd_pre_kernel<32>, dim3(grid), dim3(256), 0, s, (const bf16_t*)o, (const bf16_t*)dout, delta, B, nh, T, ldo); break;
    case 64: hipLaunchKernelGGL(attn_bwd_pre_kernel<64>, dim3(grid), dim3(256), 0, s, (const bf16_t*)o, (const bf16_t*)dout, delta, B, nh, T, ldo); break;
    case 128: hipLaunchKernelGGL(attn_bwd_pre_kernel<128>, dim3(grid), dim3(256), 0, s, (const bf16_t*)o, (const bf16_t*)dout, delta, B, nh, T, ldo); break;
    default: return (int)hipErrorInvalidValue;
  }
  ND_LAUNCH_CHECK();
}


// ---------------------------------------------------------------------------------------------
// dK, dV with LDS-DMA staging (T % 64 == 0, q/k already rotated): the Q / dO tiles and the row
// statistics of query tile it+1 move global -> LDS with global_load_lds (no VGPR round trip, no
// ds_write, no staging registers) while tile it is computed.  Row statistics come pre-negated
// (-LSE/c, -delta: attn_neg_stats_kernel) so they seed the S / dP accumulators directly.

__global__ void __launch_bounds__(256) attn_neg_stats_kernel(const float* __restrict__ lse, const float* __restrict__ delta,
                                                             float* __restrict__ nl, float* __restrict__ nd, int64_t n,
                                                             float inv_c) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    nl[i] = -lse[i] * inv_c;
    nd[i] = -delta[i];
  }
}

// NW: waves per workgroup (8 = 256-key blocks: every Q / dO tile DMA'd once per 256 keys)
// ABL (timing ablations, wrong results; ND_ATTN_DKDV_ABL): 1 no Q / dO / statistics DMA and no vmcnt wait,
// 2 no barrier, 4 no softmax VALU (P = S, dS = dP), 8 no S / dP MFMAs, 16 no dV / dK MFMAs, 32 LDS fragments
// read only in the first step
template <int N> __device__ __forceinline__ void dkdv_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }

// NB: Q / dO / statistics buffers in LDS; tile it + NB - 1 is in flight while tile it is computed
template <int HD, bool ROPE_OUT, int BQ = 64, bool PAD = false, int NW = 4, int ABL = 0, int NB = 2>
__global__ void __launch_bounds__(64 * NW, (HD >= 128 ? 1 : (HD == 64 && BQ == 64 && (ND_ATTN_X & 64)) ? 3 : 2)) attn_bwd_dkdv_dma_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const bf16_t* __restrict__ dO, const float* __restrict__ NL, const float* __restrict__ ND, bf16_t* __restrict__ dK,
    bf16_t* __restrict__ dV, int B, int nh, int nkv, int T, int64_t ld, int64_t ldo, float scale,
    const float* __restrict__ cosT, const float* __restrict__ sinT, const int* __restrict__ KS, int order) {
  constexpr int NT = HD / 16, NO = HD / 32;
  constexpr int CPR = HD / 8;              // 16-B chunks per row
  constexpr int RPI = 64 / CPR;            // rows per 1-KiB DMA wave-instruction
  constexpr int IPW = (BQ / RPI) / NW;     // DMA instructions per wave per operand tile
  constexpr int KB = 32 * NW;              // keys per workgroup
  __shared__ __attribute__((aligned(16))) bf16_t Qs[NB * BQ * HD];
  __shared__ __attribute__((aligned(16))) bf16_t dOs[NB * BQ * HD];
  __shared__ __attribute__((aligned(16))) float lse_s[NB * BQ];
  __shared__ __attribute__((aligned(16))) float del_s[NB * BQ];

  const int bk_count = B * nkv, rep = nh / nkv, nkb = (T + KB - 1) / KB;
  int kb, bk;  // see attn_bwd_dkdv_kernel
  if (order & 1) {
    const int id = xcd_remap(blockIdx.x, nkb * bk_count);
    bk = id / nkb;
    kb = id % nkb;
  } else {
    kb = (int)(blockIdx.x / bk_count);
    bk = blockIdx.x % bk_count;
  }
  const int b = bk / nkv, kvh = bk % nkv;
  const int ks = PAD ? KS[b] : 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15;
  const int kw0 = kb * KB + w * 32, key = kw0 + c32;
  const float c = scale * LOG2E;
  const bf16_t* Kb = K + (int64_t)b * T * ld + (int64_t)kvh * HD;
  const bf16_t* Vb = V + (int64_t)b * T * ld + (int64_t)kvh * HD;

  bf16x8 kf[NT], vf[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    kf[t] = key < T ? load16(Kb + (int64_t)key * ld + 16 * t + 8 * h) : zero8();
    vf[t] = key < T ? load16(Vb + (int64_t)key * ld + 16 * t + 8 * h) : zero8();
  }
  settle(kf);
  settle(vf);
  f32x16 dk[NO], dv[NO];
#pragma unroll
  for (int o = 0; o < NO; ++o) { dk[o] = f32x16{}; dv[o] = f32x16{}; }

  // per-lane DMA source offsets (constant over tiles): physical chunk p of row r carries logical
  // chunk p ^ key(r) of the soff<HD> swizzle (an XOR involution)
  const int wu = __builtin_amdgcn_readfirstlane(w);
  uint32_t vq[IPW], vd[IPW];
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int row = (wu + NW * i) * RPI + lane / CPR, p = lane % CPR;
    const int lch = (soff<HD>(row, p * 8) - row * HD) / 8;  // soff maps logical -> physical; XOR: same map back
    vq[i] = (uint32_t)(((int64_t)row * ld + lch * 8) * 2);
    vd[i] = (uint32_t)(((int64_t)row * ldo + lch * 8) * 2);
  }
  const uint32_t qs_a = lds_addr(Qs), do_a = lds_addr(dOs), ls_a = lds_addr(lse_s), ds_a = lds_addr(del_s);

  const int qstart = (kb * KB) / BQ * BQ;
  const int ntq = (T - qstart + BQ - 1) / BQ;
  const int nit = ntq * rep;
  // order bit 1: walk the query tiles from the LAST one down to the diagonal.  Every key block of a head
  // ends at query tile ntq - 1, so descending walks line the key blocks up on the SAME Q / dO tile at the
  // same step (the ascending walk starts each on its own diagonal tile: key block kb reads tile q at step
  // q - kb); with bit 0 (a head's key blocks consecutive on one XCD) the tile is then fetched once into
  // that XCD's L2 and re-read there.  Only the fp32 accumulation order of dK / dV changes.
  const bool desc = (order & 2) != 0;
  auto qtile = [&](int it) __attribute__((always_inline)) {
    const int r = it % ntq;
    return desc ? ntq - 1 - r : r;
  };
  ND_STAMP(Stamps stp; stp.start();)
  // part: 7 = everything; 1 = Q pieces, 2 = dO pieces, 4 = row statistics (ND_ATTN_X & 128 spreads them)
  auto issue = [&](int it, int part = 7) {
    const int head = kvh * rep + it / ntq;
    const int q0 = qstart + qtile(it) * BQ;
    const int buf = it % NB;
    const bf16_t* sq = Q + ((int64_t)b * T + q0) * ld + (int64_t)head * HD;
    const bf16_t* sd = dO + ((int64_t)b * T + q0) * ldo + (int64_t)head * HD;
#pragma unroll
    for (int i = 0; i < IPW; ++i) {
      const uint32_t off = (uint32_t)(buf * BQ * HD * 2 + (wu + NW * i) * 1024);
      if (part & 1) adma_b128(sq, vq[i], qs_a + off);
      if (part & 2) adma_b128(sd, vd[i], do_a + off);
    }
    ND_STAMP(stp.mark(9);)
    if ((part & 4) && wu < BQ / 64) {  // one 64-float wave-instruction per 64 rows
      const int64_t rs = ((int64_t)b * nh + head) * T + q0 + wu * 64;
      adma_b32(NL + rs, (uint32_t)(lane * 4), ls_a + (buf * BQ + wu * 64) * 4);
      adma_b32(ND + rs, (uint32_t)(lane * 4), ds_a + (buf * BQ + wu * 64) * 4);
    }
    ND_STAMP(stp.mark(8);)
  };
#pragma unroll
  for (int j = 0; j < NB - 1; ++j)
    if (j < nit) issue(j);
  bf16x8 qa[NT], da[NT], tdo[2][NO], tq[2][NO];
  bool first = true;
  constexpr bool SPREAD = (ND_ATTN_X & 128) != 0 && BQ == 128 && NB == 2;
  for (int it = 0; it < nit; ++it) {
    ND_STAMP(stp.mark(7);)
    if constexpr (!(ABL & 1)) {  // this wave's part of tile it has landed; tiles it+1 .. it+NB-2 may stay in flight
      if constexpr (NB > 2) {
        constexpr int PT = 2 * IPW;  // per tile and wave, plus 2 statistics loads on waves < BQ / 64
        if (it + NB - 2 < nit) {
          if (wu < BQ / 64) dkdv_vm<(PT + 2) * (NB - 2)>();
          else dkdv_vm<PT * (NB - 2)>();
        } else {
          dkdv_vm<0>();
        }
      } else {
        dkdv_vm<0>();
      }
    }
    ND_STAMP(stp.mark(0);)
    if constexpr (!(ABL & 2)) __syncthreads();        // everyone's; and tile it-1's buffer is free
    ND_STAMP(stp.mark(1);)
    if constexpr (!(ABL & 1) && !SPREAD) if (it + NB - 1 < nit) issue(it + NB - 1);
    const int q0 = qstart + qtile(it) * BQ;
    const int buf = it % NB;
    const bf16_t* Qt = Qs + buf * (BQ * HD);
    const bf16_t* dOt = dOs + buf * (BQ * HD);
    const float* lt = lse_s + buf * BQ;
    const float* dt = del_s + buf * BQ;
#pragma unroll
    for (int qs = 0; qs < BQ / 32; ++qs) {
      if constexpr (SPREAD && !(ABL & 1))
        if (qs < 3 && it + 1 < nit) issue(it + 1, 1 << qs);  // before the skip test: every wave issues its pieces
      const int qsub = q0 + qs * 32;
      if (kw0 > qsub + 31 || kw0 >= T) continue;  // wave-uniform: no query >= any of our keys
      // All LDS fragments of this step are issued up front (row reads for S / dP, transposing reads
      // for dV / dK) so their latency hides behind the MFMA chains and the softmax VALU instead of
      // being exposed one s_waitcnt at a time.
      ND_STAMP(stp.mark(7);)
      // ND_ATTN_X & 64 (A/B): fragments read just before their MFMAs instead, in three phases the scheduler
      // may not merge -- the register budget of 3 waves / SIMD; the partner waves cover the read latency
      constexpr bool JIT = (ND_ATTN_X & 64) != 0 && HD == 64 && BQ == 64;
      const bool rd = (!(ABL & 32) || first) && !JIT;
      first = false;
      if (rd) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          qa[t] = row_frag<HD>(Qt, qs * 32 + c32, t, h);
          da[t] = row_frag<HD>(dOt, qs * 32 + c32, t, h);
        }
      }
      f32x16 s, dp;  // seeded with -LSE / c and -delta of each query row
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int qr = qs * 32 + 8 * r4 + 4 * h;
        const float4 l4 = *reinterpret_cast<const float4*>(lt + qr);
        const float4 d4 = *reinterpret_cast<const float4*>(dt + qr);
        s[4 * r4 + 0] = l4.x; s[4 * r4 + 1] = l4.y; s[4 * r4 + 2] = l4.z; s[4 * r4 + 3] = l4.w;
        dp[4 * r4 + 0] = d4.x; dp[4 * r4 + 1] = d4.y; dp[4 * r4 + 2] = d4.z; dp[4 * r4 + 3] = d4.w;
      }
      if (rd) {
#pragma unroll
        for (int sidx = 0; sidx < 2; ++sidx)
#pragma unroll
          for (int o = 0; o < NO; ++o) {
            tdo[sidx][o] = tr_frag<HD>(dOt, qs * 32 + 16 * sidx, o * 32, g, i16);
            tq[sidx][o] = tr_frag<HD>(Qt, qs * 32 + 16 * sidx, o * 32, g, i16);
          }
      }
      ND_STAMP(stp.mark(2);)
      xprio<1>(1);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if constexpr ((ABL & 8) != 0) {
          s[t] += (float)qa[t][0];
          dp[t] += (float)da[t][0];
        } else if constexpr (JIT) {
          s = mfma32(row_frag<HD>(Qt, qs * 32 + c32, t, h), kf[t], s);
          dp = mfma32(row_frag<HD>(dOt, qs * 32 + c32, t, h), vf[t], dp);
        } else {
          s = mfma32(qa[t], kf[t], s);
          dp = mfma32(da[t], vf[t], dp);
        }
      }
      if constexpr (JIT) __builtin_amdgcn_sched_barrier(0);
      xprio<1>(0);
      ND_STAMP(stp.mark(3);)
      xprio<16>(1);
      const bool diag = (kw0 + 31 > qsub) || (qsub + 31 >= T) || (key >= T) || (PAD && kw0 < ks);
      if constexpr ((ABL & 4) != 0) {
      } else if (!diag) {
        if constexpr ((ND_ATTN_X & 2) != 0) {
          const f2v c2 = {c, c};
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            f2v x = f2v{s[r], s[r + 1]} * c2;
            x.x = fexp2(x.x);
            x.y = fexp2(x.y);
            const f2v y = x * f2v{dp[r], dp[r + 1]};
            s[r] = x.x;
            s[r + 1] = x.y;
            dp[r] = y.x;
            dp[r + 1] = y.y;
          }
        } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(s[r] * c);
          s[r] = p;
          dp[r] = p * dp[r];
        }
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qq = qsub + (r & 3) + 8 * (r >> 2) + 4 * h;
          const float p = (key <= qq && qq < T && key < T && (!PAD || key >= ks)) ? fexp2(s[r] * c) : 0.f;
          s[r] = p;
          dp[r] = p * dp[r];
        }
      }
      xprio<16>(0);
      if constexpr (JIT) __builtin_amdgcn_sched_barrier(0);
      ND_STAMP(stp.mark(4);)
      xprio<8>(1);
#pragma unroll
      for (int sidx = 0; sidx < 2; ++sidx) {
        const bf16x8 pf = pack_frag(s, sidx);
        const bf16x8 dsf = pack_frag(dp, sidx);
#pragma unroll
        for (int o = 0; o < NO; ++o) {
          if constexpr ((ABL & 16) != 0) {
            dv[o][sidx] += (float)pf[o] + (float)tdo[sidx][o][0];
            dk[o][sidx] += (float)dsf[o] + (float)tq[sidx][o][0];
          } else if constexpr (JIT) {
            dv[o] = mfma32(tr_frag<HD>(dOt, qs * 32 + 16 * sidx, o * 32, g, i16), pf, dv[o]);
            dk[o] = mfma32(tr_frag<HD>(Qt, qs * 32 + 16 * sidx, o * 32, g, i16), dsf, dk[o]);
          } else {
            dv[o] = mfma32(tdo[sidx][o], pf, dv[o]);
            dk[o] = mfma32(tq[sidx][o], dsf, dk[o]);
          }
        }
      }
      xprio<8>(0);
      ND_STAMP(stp.mark(5);)
    }
  }
  ND_STAMP(stp.mark(7);)
  if constexpr ((ABL & 1) != 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (key < T) {
    store_T<HD>(dK + ((int64_t)b * T + key) * ld + (int64_t)kvh * HD, dk, scale, h, ROPE_OUT ? cosT : nullptr, sinT, key);
    store_T<HD>(dV + ((int64_t)b * T + key) * ld + (int64_t)kvh * HD, dv, 1.f, h, nullptr, nullptr, 0);
  }
  ND_STAMP(stp.mark(6); stp.flush(1);)
}

template <int HD, bool ROPE, bool ROPE_OUT, bool PAD>
static void bwd_launch_t(const void* q, const void* k, const void* v, const void* dout, const float* lse,
                         const float* delta, void* dq, void* dk, void* dv, float* ws, int B, int nh, int nkv, int T,
                         int64_t ld, int64_t ldo, const float* cosT, const float* sinT, float scale, const int* ks,
                         hipStream_t s) {
  const int nb = (T + 127) / 128;
  const bool dma = !ROPE && ws != nullptr && T % 64 == 0 && !g_attn.dkdv_reg;
  if (dma) {
    const int64_t n = (int64_t)B * nh * T;
    float *nl = ws, *nd = ws + n;
    hipLaunchKernelGGL(attn_neg_stats_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, lse, delta, nl, nd, n,
                       1.f / (scale * LOG2E));
    if (!g_attn.dkdv_bq64 && T % 128 == 0)  // 128-query tiles when T allows (ND_DKDV_BQ=64: 64, A/B)
      hipLaunchKernelGGL((attn_bwd_dkdv_dma_kernel<HD, ROPE_OUT, 128, PAD>), dim3(nb * B * nkv), dim3(256), 0, s,
                         (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, nl, nd,
                         (bf16_t*)dk, (bf16_t*)dv, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, ks, dkdv_order(nh, nkv));
    else
      hipLaunchKernelGGL((attn_bwd_dkdv_dma_kernel<HD, ROPE_OUT, 64, PAD>), dim3(nb * B * nkv), dim3(256), 0, s,
                         (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, nl, nd,
                         (bf16_t*)dk, (bf16_t*)dv, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, ks, dkdv_order(nh, nkv));
  } else {
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD, ROPE, ROPE_OUT, PAD>), dim3(nb * B * nkv), dim3(256), 0, s,
                       (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, lse, delta,
                       (bf16_t*)dk, (bf16_t*)dv, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, ks, dkdv_order(nh, nkv));
  }
  if (dma)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, ROPE, ROPE_OUT, !ROPE, false, PAD>), dim3(nb * B * nh), dim3(256), 0, s,
                       (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, lse, delta,
                       (bf16_t*)dq, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, nullptr, nullptr, nullptr, ks, attn_order());
  else
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, ROPE, ROPE_OUT, false, false, PAD>), dim3(nb * B * nh), dim3(256), 0, s, (const bf16_t*)q,
                       (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, lse, delta, (bf16_t*)dq, B, nh, nkv,
                       T, ld, ldo, scale, cosT, sinT, nullptr, nullptr, nullptr, ks, attn_order());
}

// rope_mode 0: no RoPE; 1: q/k are RAW projections -- rotated on load, dq/dk un-rotated on store;
// 2: q/k were rotated in place before the forward -- only the dq/dk un-rotation (store epilogue).
template <int HD>
static int bwd_launch(const void* q, const void* k, const void* v, const void* dout, const float* lse, const float* delta,
                      void* dq, void* dk, void* dv, float* ws, int B, int nh, int nkv, int T, int64_t ld, int64_t ldo,
                      const float* cosT, const float* sinT, float scale, int rope_mode, const int* ks, hipStream_t s) {
  if (rope_mode == 1)
    (ks ? bwd_launch_t<HD, true, true, true> : bwd_launch_t<HD, true, true, false>)(q, k, v, dout, lse, delta, dq, dk, dv, ws, B, nh, nkv, T, ld, ldo, cosT, sinT, scale, ks, s);
  else if (rope_mode == 2)
    (ks ? bwd_launch_t<HD, false, true, true> : bwd_launch_t<HD, false, true, false>)(q, k, v, dout, lse, delta, dq, dk, dv, ws, B, nh, nkv, T, ld, ldo, cosT, sinT, scale, ks, s);
  else
    (ks ? bwd_launch_t<HD, false, false, true> : bwd_launch_t<HD, false, false, false>)(q, k, v, dout, lse, delta, dq, dk, dv, ws, B, nh, nkv, T, ld, ldo, cosT, sinT, scale, ks, s);
  ND_LAUNCH_CHECK();
}

// dq/dk/dv may point into one packed dqkv buffer (row stride ld).  ks: see nd_attn_fwd_ks.
ND_API int nd_attn_bwd_ks(const void* q, const void* k, const void* v, const void* dout, const float* lse,
                          const float* delta, void* dq, void* dk, void* dv, float* ws, int B, int nh, int nkv,
                          int T, int hd, int64_t ld, int64_t ldo, const float* cosT, const float* sinT, float scale,
                          int rope_mode, const int* ks, hipStream_t s) {
  if (nh % nkv || (ld % 8) || (ldo % 8)) return (int)hipErrorInvalidValue;
  if (rope_mode && !(cosT && sinT)) return (int)hipErrorInvalidValue;
  switch (hd) {
    case 32: return bwd_launch<32>(q, k, v, dout, lse, delta, dq, dk, dv, ws, B, nh, nkv, T, ld, ldo, cosT, sinT, scale, rope_mode, ks, s);
    case 64: return bwd_launch<64>(q, k, v, dout, lse, delta, dq, dk, dv, ws, B, nh, nkv, T, ld, ldo, cosT, sinT, scale, rope_mode, ks, s);
    case 128: return bwd_launch<128>(q, k, v, dout, lse, delta, dq, dk, dv, ws, B, nh, nkv, T, ld, ldo, cosT, sinT, scale, rope_mode, ks, s);
    default: return (int)hipErrorInvalidValue;
  }
}

ND_API int nd_attn_bwd(const void* q, const void* k, const void* v, const void* dout, const float* lse,
                       const float* delta, void* dq, void* dk, void* dv, float* ws, int B, int nh, int nkv,
                       int T, int hd, int64_t ld, int64_t ldo, const float* cosT, const float* sinT, float scale,
                       int rope_mode, hipStream_t s) {
  return nd_attn_bwd_ks(q, k, v, dout, lse, delta, dq, dk, dv, ws, B, nh, nkv, T, hd, ld, ldo, cosT, sinT, scale,
                        rope_mode, nullptr, s);
}

// Backward with the row statistics fused into the dQ kernel (PRE): dQ (writes -delta, -LSE/c into
// ws) -> dK/dV; no attn_bwd_pre / attn_neg_stats passes.  LDS-DMA kernels only: q/k already rotated
// (rope_mode 0 or 2), T % 64 == 0.  ws: 2 * B * nh * T floats.
template <int HD, bool ROPE_OUT, bool PAD>
static int bwd_fused_launch(const void* q, const void* k, const void* v, const void* o, const void* dout,
                            const float* lse, void* dq, void* dk, void* dv, float* ws, int B, int nh, int nkv, int T,
                            int64_t ld, int64_t ldo, const float* cosT, const float* sinT, float scale, const int* ks,
                            hipStream_t s) {
  const int nb = (T + 127) / 128;
  const int64_t n = (int64_t)B * nh * T;
  float *nl = ws, *nd = ws + n;
  bool done = false;
  if constexpr (HD >= 64) {  // ND_ATTN_DQ_W=8: 256-query blocks
    if (!done && g_attn.dq_w8) {
      hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, false, ROPE_OUT, true, true, PAD, 8>), dim3((T + 255) / 256 * B * nh),
                         dim3(512), 0, s, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout,
                         lse, nullptr, (bf16_t*)dq, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, (const bf16_t*)o, nl, nd,
                         ks, attn_order());
      done = true;
    }
  }
  if (!done)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, false, ROPE_OUT, true, true, PAD>), dim3(nb * B * nh), dim3(256), 0, s,
                       (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, lse, nullptr,
                       (bf16_t*)dq, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, (const bf16_t*)o, nl, nd, ks, attn_order());
  bool kw8 = false;
  if constexpr (HD >= 64) kw8 = g_attn.dkdv_w8 && T % 128 == 0;
  if (kw8)  // 256-key blocks
    hipLaunchKernelGGL((attn_bwd_dkdv_dma_kernel<HD, ROPE_OUT, 128, PAD, 8>), dim3((T + 255) / 256 * B * nkv), dim3(512),
                       0, s, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, nl, nd,
                       (bf16_t*)dk, (bf16_t*)dv, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, ks, dkdv_order(nh, nkv));
  else if (const int nbv = g_attn.dkdv_nb) {  // 64-query tiles, A/B
#define ND_DN(X) hipLaunchKernelGGL((attn_bwd_dkdv_dma_kernel<HD, ROPE_OUT, 64, PAD, 4, 0, X>), dim3(nb * B * nkv), dim3(256), \
      0, s, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, nl, nd, (bf16_t*)dk, (bf16_t*)dv, \
      B, nh, nkv, T, ld, ldo, scale, cosT, sinT, ks, dkdv_order(nh, nkv))
    if (nbv == 2) ND_DN(2);
    else if (nbv == 3) ND_DN(3);
    else ND_DN(4);
#undef ND_DN
  } else if (T % 128 == 0 && !(ND_ATTN_X & 64)) {
    switch (g_attn.dkdv_abl) {  // always 0 outside an ND_ABLATION build
#ifdef ND_ABLATION
#define ND_DA(X) case X: hipLaunchKernelGGL((attn_bwd_dkdv_dma_kernel<HD, ROPE_OUT, 128, PAD, 4, X>), dim3(nb * B * nkv), \
      dim3(256), 0, s, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, nl, nd, (bf16_t*)dk, \
      (bf16_t*)dv, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, ks, dkdv_order(nh, nkv)); break;
      ND_DA(1) ND_DA(2) ND_DA(3) ND_DA(4) ND_DA(8) ND_DA(16) ND_DA(24) ND_DA(32) ND_DA(28) ND_DA(63)
#undef ND_DA
#endif
      default:
        hipLaunchKernelGGL((attn_bwd_dkdv_dma_kernel<HD, ROPE_OUT, 128, PAD>), dim3(nb * B * nkv), dim3(256), 0, s,
                           (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, nl, nd,
                           (bf16_t*)dk, (bf16_t*)dv, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, ks, dkdv_order(nh, nkv));
    }
  } else
    hipLaunchKernelGGL((attn_bwd_dkdv_dma_kernel<HD, ROPE_OUT, 64, PAD>), dim3(nb * B * nkv), dim3(256), 0, s,
                       (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, (const bf16_t*)dout, nl, nd,
                       (bf16_t*)dk, (bf16_t*)dv, B, nh, nkv, T, ld, ldo, scale, cosT, sinT, ks, dkdv_order(nh, nkv));
  ND_LAUNCH_CHECK();
}

ND_API int nd_attn_bwd_fused_ks(const void* q, const void* k, const void* v, const void* o, const void* dout,
                                const float* lse, void* dq, void* dk, void* dv, float* ws, int B, int nh, int nkv,
                                int T, int hd, int64_t ld, int64_t ldo, const float* cosT, const float* sinT,
                                float scale, int rope_mode, const int* ks, hipStream_t s) {
  if (nh % nkv || (ld % 8) || (ldo % 8) || T % 64 || ws == nullptr || rope_mode == 1) return (int)hipErrorInvalidValue;
  if (rope_mode == 2 && !(cosT && sinT)) return (int)hipErrorInvalidValue;
  switch (hd) {
#define ND_BF(H)                                                                                               \
  case H:                                                                                                      \
    return rope_mode == 2 ? (ks ? bwd_fused_launch<H, true, true> : bwd_fused_launch<H, true, false>)(q, k, v, o, dout, lse, dq, dk, dv, ws, B, nh, nkv, T, ld, \
                                                      ldo, cosT, sinT, scale, ks, s)                           \
                          : (ks ? bwd_fused_launch<H, false, true> : bwd_fused_launch<H, false, false>)(q, k, v, o, dout, lse, dq, dk, dv, ws, B, nh, nkv, T, ld, \
                                                       ldo, cosT, sinT, scale, ks, s);
    ND_BF(32)
    ND_BF(64)
    ND_BF(128)
#undef ND_BF
    default: return (int)hipErrorInvalidValue;
  }
}

ND_API int nd_attn_bwd_fused(const void* q, const void* k, const void* v, const void* o, const void* dout,
                             const float* lse, void* dq, void* dk, void* dv, float* ws, int B, int nh, int nkv, int T,
                             int hd, int64_t ld, int64_t ldo, const float* cosT, const float* sinT, float scale,
                             int rope_mode, hipStream_t s) {
  return nd_attn_bwd_fused_ks(q, k, v, o, dout, lse, dq, dk, dv, ws, B, nh, nkv, T, hd, ld, ldo, cosT, sinT, scale,
                              rope_mode, nullptr, s);
}
