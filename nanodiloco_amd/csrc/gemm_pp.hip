// Ping-pong projection GEMM for gfx950 (round 3): C[M, N] = A[M, K] . B[N, K]^T, bf16 in, fp32
// accumulate -- the forward and input-gradient GEMMs of every Llama projection (B = W[out, in], or its
// transposed copy W^T[in, out] for dgrad) and the lm-head logits / dgrad.
//
// Why a new structure (docs/DESIGN.md §3): the round-2 four-wave kernel (one MFMA wave per SIMD)
// stalls its matrix pipe whenever its only wave waits on LDS reads, LDS-DMA issue or a barrier
// (43 % MFMA busy vs hipBLASLt's 63 %).  Here every SIMD holds TWO waves with opposite roles:
//
//   * 512 threads = 8 waves = two groups of four; waves 0-3 (group 0) and 4-7 (group 1) each cover all
//     four SIMDs once, so every SIMD pairs one wave of each group (MI355X_MICROARCH "Two waves per
//     SIMD", item 9: split roles by wave number >= 4).
//   * 256 x 256 output tile, BK = 64; group g owns tile rows 128 g .. 128 g + 127, wave w & 3 owns
//     64 columns: 128 x 64 per wave = 8 x 4 v_mfma_f32_16x16x32_bf16 accumulators (128 AGPRs) plus
//     one K-tile of fragments (8 + 4 blocks x 2 k-steps of bf16x8 = 96 VGPRs): 2 waves / SIMD.
//   * Each K-tile is two phases per group, LOAD (all 24 ds_read_b128 fragment reads of the K-tile,
//     this group's LDS-DMA pieces, lgkmcnt(0)) and COMPUTE (64 MFMAs from registers), and group 1 runs
//     ONE BARRIER BEHIND group 0:
//
//         barrier:      ... | 2s      | 2s+1       | 2s+2       | ...
//         group 0:          LOAD(s)   COMPUTE(s)   LOAD(s+1)
//         group 1:          COMPUTE(s-1) LOAD(s)   COMPUTE(s)
//
//     so while one wave of a SIMD issues its MFMA chain (s_setprio 1) its partner issues the loads of
//     the other half of the tile: the matrix pipe never waits for LDS, DMA issue or the barrier.
//
// LDS: two 64-KiB K-tile buffers of four 16-KiB half-tiles (A0 = tile rows 0-127, A1 = 128-255, B0, B1),
// [128 rows][64 k] with the 16-B chunk index XOR-swizzled by (row >> 1) & 7 (on the DMA SOURCE
// address -- LDS-DMA writes lane-linear -- and on the ds_read_b128 reads): every 16-lane group of a
// fragment read hits 16 distinct bank slots.  DMA ownership (derived from the phase table above,
// each buffer restaged only after both groups' reads of it have retired):
//
//   group 0, LOAD(s): B0 + B1 of K-tile s+1   (8 pieces / wave; retired by vmcnt at the end of
//                                              its COMPUTE(s), read from LOAD(s+1) on)
//   group 1, LOAD(s): A1 of K-tile s+1, then A0 of K-tile s+2 (4 + 4 pieces / wave; A1(s+1) retired
//                     at the end of its COMPUTE(s), A0(s+2) at the end of its LOAD(s+1))
//
// The waits are counted (`s_waitcnt vmcnt(N)`, never a drain of the whole stream).  Half-tiles whose rows
// all exist are staged with FLAT-global LDS loads (`global_load_lds_dwordx4`, SGPR base + per-lane offset;
// round 4, 1.004-1.011x); tail half-tiles go through buffer descriptors whose record count ends at the
// operand's last row, so the M / N tail rows read as out-of-range (no clamping, tile-independent per-lane
// offsets).
//
// Persistent: one workgroup per CU walks tiles first, first + G, ... (XCD-remapped; GM m-panels per
// group of tiles so one XCD's 32 concurrent tiles share A / B panels in its L2), and the K-tile
// stream -- DMA, fragment reads, MFMAs -- runs across tile boundaries.  A tile's epilogue (fused
// variants below) is issued inside the next tile's first LOAD phase, behind that phase's DMA, with
// 16-B buffer stores the counted waits leave in flight.
//
// Fused epilogues (each removes a separate HBM round trip of the [M, N] output):
//   PP_STORE    C = bf16(acc)
//   PP_ROPE     q|k|v projection: RoPE (half-split, head_dim HD = 32 / 64) on the q and k columns of
//               the fp32 accumulator before the one bf16 rounding; v columns stored plainly
//   PP_SWIGLU   gate|up projection, 128 gate / up units per tile (wave column group = 32 gate rows
//               then the 32 matching up rows of the weight): stores gu = [gate | up] AND
//               act = silu(gate) * up
//   PP_DSWIGLU  down-projection input gradient: acc = d(act); reads gate / up, stores d(gate | up)
//
// fp8 operands (round 4, template F8): the same kernel with a 128-element fp8 K-tile (the same 128-B LDS
// rows), one v_mfma_scale_f32_16x16x128_f8f6f4 per fragment pair, every epilogue on acc * sa * sb; the Q
// forms of the SwiGLU epilogues write the e4m3 act / e5m2 d(gate|up) instead of the bf16 tensors
// (profiles/r4_fp8_pp.md).
//
// Reference role: every nn.Linear of HF LlamaForCausalLM (/root/reference/nanodiloco/main.py:97-99,
// run at :109-111).
#include "common.h"
#include <cstdlib>
#include <type_traits>

using namespace nd;

namespace {
typedef __bf16 bfv8 __attribute__((ext_vector_type(8)));
constexpr int TM = 256, TN = 256, TK = 64;
constexpr uint32_t HALF_B = 128 * TK * 2;  // bytes of one half-tile (16 KiB)
constexpr uint32_t BUF_B = 4 * HALF_B;     // bytes of one K-tile buffer (64 KiB)
constexpr int LGKM0 = 0xC07F;              // s_waitcnt lgkmcnt(0), vmcnt / expcnt at their maxima

enum : int { PP_STORE = 0, PP_ROPE = 1, PP_SWIGLU = 2, PP_DSWIGLU = 3 };
#ifndef ND_MLP_COEF_DEFAULT
#define ND_MLP_COEF_DEFAULT 1  // saved-tensor form of the fused SwiGLU pair (g_mlp_coef below): the coefficient form
                               // (down dgrad + SwiGLU backward 1.046x, step +0.2 %: profiles/r6_mlp_coef_ab.md)
#endif

struct PPEpi {
  const float* cosT;  // PP_ROPE: fp32 [T, hd] tables (HF cat(freqs, freqs) layout)
  const float* sinT;
  int T, rope_cols;
  bf16_t* act;        // PP_SWIGLU: act [M, F]
  int64_t ld_act;
  const bf16_t* gu;   // PP_DSWIGLU: gu [M, 2F]
  int64_t ld_gu;
  const float* sa;    // fp8 operands (F8 != 0): per-tensor dequantisation scales, acc *= sa[0] * sb[0]
  const float* sb;
  uint8_t* q8;          // Q: fp8 output INSTEAD of the bf16 act (PP_SWIGLU, e4m3) / d(gate|up) (PP_DSWIGLU, e5m2)
  int64_t ld_q8;
  const float* qscale;  // delayed-scaling scale of that output (device scalar)
  float* qamax;         // amax partial slots (float bits as ordered ints)
  int qparts;
};

// stores per wave per tile epilogue (counted by the vmcnt waits that follow it)
template <int EPI> struct NStores { static constexpr int v = EPI == PP_SWIGLU ? 24 : EPI == PP_DSWIGLU ? 32 : 16; };
#ifndef DSW_PF
#define DSW_PF 6  // PP_DSWIGLU epilogue: gate / up load steps in flight
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// one LDS-DMA wave-instruction: 64 lanes x 16 B from descriptor r at per-lane byte offset voff to
// LDS [lds, lds + 1 KiB); lanes past the descriptor's record count read nothing (tail rows)
__device__ __forceinline__ void dma(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds) : "memory");
}
// FLAT-global form (SGPR base + 32-bit per-lane offset, no range check): the default for half-tiles whose rows
// all exist (tail half-tiles keep the range-checked buffer form)
__device__ __forceinline__ void gdma(const void* base, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(base), "s"(lds) : "memory");
}
// accumulator pinned to AGPRs (tied operand): the chain on one accumulator needs no wait states;
// compiler code reading the result waits for drain()
#ifndef ND_PP_ASM_MFMA
__device__ __forceinline__ void mma(const bf16x8& a, const bf16x8& b, f32x4& c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0, 0);
}
__device__ __forceinline__ void mma0(const bf16x8& a, const bf16x8& b, f32x4& c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
}
#else
__device__ __forceinline__ void mma(const bf16x8& a, const bf16x8& b, f32x4& c) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
// first k-step of a tile: zero accumulator input (no per-tile AGPR zeroing)
__device__ __forceinline__ void mma0(const bf16x8& a, const bf16x8& b, f32x4& c) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
}
#endif
// fp8 operands (F8 1: A e4m3, B e4m3; 2: A e5m2, B e4m3): one 16x16x128 MFMA on the two 16-B halves of
// each fragment (the lane's 32 K bytes), unit E8M0 block scales (`one` = 0x7F7F7F7F).  The MFMA's first
// source is B (cbsz = B's format), its second A (blgp = A's format).
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ i32x8 cat16(const bf16x8& x, const bf16x8& y) {
  const i32x4 a = __builtin_bit_cast(i32x4, x), b = __builtin_bit_cast(i32x4, y);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
template <int F8>
__device__ __forceinline__ void mma8(const i32x8& b, const i32x8& a, f32x4& c, int one) {
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a, c, 0, F8 == 1 ? 0 : 1, 0, one, 0, one);
}
template <int F8>
__device__ __forceinline__ void mma8z(const i32x8& b, const i32x8& a, f32x4& c, int one) {
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a, f32x4{0.f, 0.f, 0.f, 0.f}, 0, F8 == 1 ? 0 : 1, 0, one, 0,
                                                         one);
}
__device__ __forceinline__ void drain() { asm volatile("s_nop 15\n\ts_nop 3" ::: "memory"); }
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}
template <int N> __device__ __forceinline__ void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }
// runtime count out of a small compile-time set (wave-uniform branch)
template <int NST> __device__ __forceinline__ void vmwait_n(int n) {
  switch (n) {
    case 0: vmwait<0>(); break;
    case 4: vmwait<4>(); break;
    case 8: vmwait<8>(); break;
    case NST: vmwait<NST>(); break;
    case NST + 4: vmwait<NST + 4>(); break;
    case NST + 8: vmwait<NST + 8>(); break;
    default: vmwait<0>(); break;
  }
}

// bf16-pack the 4-column quads of two adjacent 16-column blocks (x = block b, y = block b + 1) and
// v_permlane16_swap them: lane row q = lane >> 4 then holds 8 consecutive columns
// (block b + (q & 1), columns 8 (q >> 1) .. + 7) -> one 16-B store
__device__ __forceinline__ u32x4 pair16(const f32x4& x, const f32x4& y) {
  const auto s0 = __builtin_amdgcn_permlane16_swap(pack2(x[0], x[1]), pack2(y[0], y[1]), false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(pack2(x[2], x[3]), pack2(y[2], y[3]), false, false);
  u32x4 d = u32x4{s0[0], s1[0], s0[1], s1[1]};
  asm volatile("s_nop 1" : "+v"(d));  // permlane result -> store data: two wait states
  return d;
}
__device__ __forceinline__ float rbf(float x) { return lo_bf(pack2(x, 0.f)); }
__device__ __forceinline__ float silu(float g) { return g * fast_sigmoid(g); }

// ---- epilogue of one tile: the wave's 128 x 64 accumulator block (rows 128 g + .., columns 64 wn + ..)
// of the tile at (m0, n0) -> the fused output(s).  Exactly NStores<EPI> 16-B buffer stores per wave
// (the callers' counted waits rely on it); out-of-range lanes drop through the descriptor's record
// count or an offset sentinel.  `smem` + 2 BUF_B + 4 KiB w: the wave's private C staging region.
// FORM (PP_SWIGLU / PP_DSWIGLU only, round 6): 0 -- the forward keeps gu = [gate | up] for the backward, which
// recomputes sigmoid(gate) and the SwiGLU derivative per element; 1 (coefficient form) -- the forward, which has
// sigmoid(gate) in hand for act, keeps [A | B] instead, A = up s (1 + gate (1 - s)) = d act / d gate and
// B = gate s = d act / d up (s = sigmoid(gate), all from the bf16-rounded gate / up act is computed from), so the
// backward epilogue is d(gate) = d(act) A, d(up) = d(act) B: two multiplies per unit instead of a sigmoid and ten
// more VALU.  Same buffer, same traffic; the two launchers read one switch (g_mlp_coef) so they always agree.
template <int EPI, int HD, int ABL, int F8 = 0, int Q = 0, int FORM = 0>
__device__ __forceinline__ void pp_epilogue(const f32x4 (&acc)[8][4], bf16_t* __restrict__ C, int M, int N,
                                            int64_t ldc, const PPEpi& ep, int m0, int n0, int g, int wn, int w,
                                            int lane, char* smem, float sc, float qs, float& qmax) {
  // store cache policy: nt (aux 2) by default, plain with ABL 32; ABL 2048 adds sc1 (aux 16), whose stores do not
  // keep the written line in the XCD's L2 (MI355X_MICROARCH store flavours) -- A/B of L2 room for the K-loop
  constexpr int STP = ((ABL & 32) ? 0 : 2) | ((ABL & 2048) ? 16 : 0);
  // the SwiGLU forward's direct (half-line) stores: plain policy by default; ABL 512 (A/B) nt like the staged ones
  constexpr int SWP = ((ABL & 2048) ? 16 : 0) | ((ABL & 512) ? 2 : 0);

    // per-lane row offsets derive from an opaque zero: otherwise LICM hoists every row's store
    // offset out of the tile loop and keeps ~16 VGPRs live through the whole K-loop (spills)
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    const int r16 = (lane & 15) + z, q = (lane >> 4) + z;
    if constexpr ((ABL & 128) != 0) m0 = n0 = 0;  // ablation: every tile stores over tile 0 (L2-resident)
    const int rows = M - m0 < TM ? M - m0 : TM;
    if constexpr (EPI == PP_STORE || EPI == PP_ROPE) {
      const auto cr = rsrc(C + (int64_t)m0 * ldc, (uint32_t)((int64_t)rows * ldc * 2));
      constexpr int HALFD = HD / 2;
      // RoPE tables: the loads of four row blocks are issued together (64 VGPRs -- the next K-tile's
      // fragment registers are free during the epilogue), so the epilogue waits for table data twice
      // per tile instead of once per row block (each wait also drains the LDS-DMA issued before it)
      constexpr int NJ = EPI == PP_ROPE ? (HALFD + 15) / 16 : 1;
      float4 ctab[4][NJ], stab[4][NJ];
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const int mr = g * 128 + a * 16 + r16;  // row inside the tile
        if constexpr (EPI == PP_ROPE) {
          if ((a & 3) == 0) {
#pragma unroll
            for (int aa = 0; aa < 4; ++aa) {
              const int t = (m0 + mr + aa * 16) % ep.T;
#pragma unroll
              for (int j = 0; j < NJ; ++j) {
                if constexpr ((ABL & 16384) != 0) {  // ablation: no table loads (wrong result, timing only)
                  ctab[aa][j] = float4{0.5f, 0.25f, (float)t, (float)j};
                  stab[aa][j] = float4{(float)q, 0.125f, 0.75f, (float)aa};
                  continue;
                }
                ctab[aa][j] = *reinterpret_cast<const float4*>(ep.cosT + (int64_t)t * HD + j * 16 + 4 * q);
                stab[aa][j] = *reinterpret_cast<const float4*>(ep.sinT + (int64_t)t * HD + j * 16 + 4 * q);
              }
            }
          }
        }
        f32x4 v[4] = {acc[a][0], acc[a][1], acc[a][2], acc[a][3]};
        if constexpr (F8 != 0) {
#pragma unroll
          for (int b = 0; b < 4; ++b) v[b] *= sc;
        }
        if constexpr (EPI == PP_ROPE) {
          // the wave's 64 columns are one 64-wide head (or two 32-wide ones): column block b pairs
          // with b + HD / 32 in the same lane.  Only q / k waves get here (pp_epilogue_any: v waves run
          // the plain store epilogue), so no per-element selects
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            if (((b * 16) % HD) >= HALFD) continue;
            const int p = b + HALFD / 16, j = ((b * 16) % HD) / 16;
            const float4 c = ctab[a & 3][j], s = stab[a & 3][j];
            const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float x1 = v[b][r], x2 = v[p][r];
              v[b][r] = x1 * cc[r] - x2 * ss[r];
              v[p][r] = x2 * cc[r] + x1 * ss[r];
            }
          }
        }
        if constexpr ((ABL & 256) == 0) {
          // full-line stores: two row blocks (32 rows x 128 B) through the wave's private 4-KiB LDS
          // staging region (behind the K-tile buffers; 16-B chunk index ^ (row & 7)), read back
          // as whole rows -- each buffer_store then writes 8 full 128-B lines instead of 16 halves
          char* st = smem + 2 * BUF_B + w * 4096;
          const int row = (a & 1) * 16 + r16;
#pragma unroll
          for (int bp = 0; bp < 2; ++bp) {
            const int ch = (2 * bp + (q & 1)) * 2 + (q >> 1);
            *reinterpret_cast<u32x4*>(st + row * 128 + ((ch ^ (row & 7)) << 4)) = pair16(v[2 * bp], v[2 * bp + 1]);
          }
          if (a & 1) {
            asm volatile("" ::: "memory");
            const int lc = (lane + z) & 7;
            const int col = n0 + wn * 64 + lc * 8;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int rr = i * 8 + ((lane + z) >> 3);
              const u32x4 d = *reinterpret_cast<const u32x4*>(st + rr * 128 + ((lc ^ (rr & 7)) << 4));
              const int gr = g * 128 + (a - 1) * 16 + rr;
              // ABL 8192 (ablation builds): every store out of range -- the epilogue's instructions without its HBM writes
              const uint32_t off = col < N && (ABL & 8192) == 0 ? (uint32_t)(((int64_t)gr * ldc + col) * 2) : 0x80000000u;
              __builtin_amdgcn_raw_buffer_store_b128(d, cr, off, 0, STP);
            }
            asm volatile("" ::: "memory");
          }
        } else {
#pragma unroll
          for (int bp = 0; bp < 2; ++bp) {
            const int col = n0 + wn * 64 + (2 * bp + (q & 1)) * 16 + (q >> 1) * 8;
            const uint32_t off = col < N ? (uint32_t)(((int64_t)mr * ldc + col) * 2) : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b128(pair16(v[2 * bp], v[2 * bp + 1]), cr, off, 0, STP);
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // one row block at a time: bounded epilogue registers
      }
    } else if constexpr (EPI == PP_SWIGLU) {
      // lane's gate units f = n0 + 32 wn + 16 b + 4 q + r (b = 0, 1) pair with up = acc[a][b + 2]
      const auto cr = rsrc(C + (int64_t)m0 * ldc, (uint32_t)((int64_t)rows * ldc * 2));
      const auto ar = rsrc(ep.act + (int64_t)m0 * ep.ld_act, (uint32_t)((int64_t)rows * ep.ld_act * 2));
      const int f = n0 + wn * 32 + (q & 1) * 16 + (q >> 1) * 8;
      const bool ok = f < N;
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const int mr = g * 128 + a * 16 + r16;
        f32x4 g2[2], u2[2], y2[2];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            g2[j][r] = rbf(F8 != 0 ? acc[a][j][r] * sc : acc[a][j][r]);  // act from the rounded gate / up: what the backward reads
            u2[j][r] = rbf(F8 != 0 ? acc[a][j + 2][r] * sc : acc[a][j + 2][r]);
            if constexpr (FORM == 1) {
              const float sg = fast_sigmoid(g2[j][r]), sl = g2[j][r] * sg;  // sl = silu(gate), bitwise silu()
              y2[j][r] = sl * u2[j][r];
              const float cg = (u2[j][r] * sg) * (1.f + g2[j][r] * (1.f - sg));  // A (stored where gate was)
              g2[j][r] = cg;
              u2[j][r] = sl;                                                   // B (stored where up was)
            } else {
              y2[j][r] = silu(g2[j][r]) * u2[j][r];
            }
          }
        const bool okst = ok && (ABL & 8192) == 0;  // ABL 8192: stores out of range (no HBM writes; timing only)
        const uint32_t og = okst ? (uint32_t)(((int64_t)mr * ldc + f) * 2) : 0x80000000u;
        const uint32_t ou = okst ? (uint32_t)(((int64_t)mr * ldc + N + f) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(pair16(g2[0], g2[1]), cr, og, 0, SWP);
        __builtin_amdgcn_raw_buffer_store_b128(pair16(u2[0], u2[1]), cr, ou, 0, SWP);
        if constexpr (Q != 0) {
          // e4m3 act (bitwise a separate cast of the bf16 act, which is not written): the lane's 8 units in
          // column order (pair16's permutation on the fp32 values), bf16-rounded, scaled, one 8-B store
          const auto qr = rsrc(ep.q8 + (int64_t)m0 * ep.ld_q8, (uint32_t)((int64_t)rows * ep.ld_q8));
          float e[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(y2[0][r]), __float_as_uint(y2[1][r]),
                                                              false, false);
            e[r] = rbf(__uint_as_float(sw[0]));
            e[4 + r] = rbf(__uint_as_float(sw[1]));
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) qmax = fmaxf(qmax, fabsf(e[j]));
          const uint2 o = uint2{cvt4<0>(e[0] * qs, e[1] * qs, e[2] * qs, e[3] * qs),
                                cvt4<0>(e[4] * qs, e[5] * qs, e[6] * qs, e[7] * qs)};
          const uint32_t oq = ok ? (uint32_t)((int64_t)mr * ep.ld_q8 + f) : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, o), qr, oq, 0, 0);
        } else {
          const uint32_t oy = okst ? (uint32_t)(((int64_t)mr * ep.ld_act + f) * 2) : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b128(pair16(y2[0], y2[1]), ar, oy, 0, SWP);
        }
      }
    } else {  // PP_DSWIGLU: acc = d(act)[m][f]; C = d(gate | up) [M, 2N]
      const auto cr = rsrc(C + (int64_t)m0 * ldc, (uint32_t)((int64_t)rows * ldc * 2));
      const auto gr = rsrc(ep.gu + (int64_t)m0 * ep.ld_gu, (uint32_t)((int64_t)rows * ep.ld_gu * 2));
      // the 16 (row block, column pair) steps read gate / up from HBM: their loads run PF steps ahead
      // (2 x PF x 4 VGPRs, taken from the next K-tile's fragment registers, free here) instead of one
      // -- one exposed HBM round trip per tile instead of per step
      constexpr int PF = Q != 0 ? 4 : DSW_PF;  // the fp8-output form needs the registers
      u32x4 gq[PF], uq[PF];
      auto gu_off = [&](int st, int half) -> uint32_t {
        const int a = st >> 1, bp = st & 1;
        const int mr = g * 128 + a * 16 + r16;
        const int f = n0 + wn * 64 + (2 * bp + (q & 1)) * 16 + (q >> 1) * 8;
        // branch-free select (a ?: here becomes two exec-masked copies of the load)
        const uint32_t okm = 0u - (uint32_t)(f < N);
        return ((uint32_t)(((int64_t)mr * ep.ld_gu + half * N + f) * 2) & okm) | (0x80000000u & ~okm);
      };
#pragma unroll
      for (int st = 0; st < PF; ++st) {
        if constexpr ((ABL & 4096) != 0) {  // ablation: no gate / up loads (wrong result)
          gq[st] = u32x4{(uint32_t)lane, 1u, 2u, 3u};
          uq[st] = u32x4{3u, 2u, 1u, (uint32_t)lane};
          continue;
        }
        gq[st] = __builtin_amdgcn_raw_buffer_load_b128(gr, gu_off(st, 0), 0, 0);
        uq[st] = __builtin_amdgcn_raw_buffer_load_b128(gr, gu_off(st, 1), 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch above the first use (the scheduler sinks it)
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const int mr = g * 128 + a * 16 + r16;
#pragma unroll
        for (int bp = 0; bp < 2; ++bp) {
          // after the pair swap this lane holds d(act) of 8 consecutive units f .. f + 7
          const int f = n0 + wn * 64 + (2 * bp + (q & 1)) * 16 + (q >> 1) * 8;
          const bool ok = f < N;
          const int st = 2 * a + bp;
          const u32x4 gv = gq[st % PF], uv = uq[st % PF];
          if (st + PF < 16 && (ABL & 4096) == 0) {
            gq[st % PF] = __builtin_amdgcn_raw_buffer_load_b128(gr, gu_off(st + PF, 0), 0, 0);
            uq[st % PF] = __builtin_amdgcn_raw_buffer_load_b128(gr, gu_off(st + PF, 1), 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
          // d(act) as fp32 in the same 8-unit order: swap the fp32 quads like pair16 does
          f32x4 d0, d1;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[a][2 * bp][r]),
                                                              __float_as_uint(acc[a][2 * bp + 1][r]), false, false);
            d0[r] = __uint_as_float(sw[0]);
            d1[r] = __uint_as_float(sw[1]);
            if constexpr (F8 != 0) {
              d0[r] *= sc;
              d1[r] *= sc;
            }
          }
          // lane row q even: d0 = units 0-3, d1 = units 4-7 of block 2 bp (cols 8 (q >> 1) ..);
          // odd: d0 = block 2 bp + 1's units 0-3 ... -- the same (x, y) order pair16 packs
          float dg[8], du[8];
          const uint32_t gw[4] = {gv[0], gv[1], gv[2], gv[3]}, uw[4] = {uv[0], uv[1], uv[2], uv[3]};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = e < 4 ? d0[e] : d1[e - 4];
            const float gg = (e & 1) ? hi_bf(gw[e >> 1]) : lo_bf(gw[e >> 1]);
            const float uu = (e & 1) ? hi_bf(uw[e >> 1]) : lo_bf(uw[e >> 1]);
            if constexpr (FORM == 1) {  // gg = A, uu = B (coefficient form, see pp_epilogue)
              dg[e] = d * gg;
              du[e] = d * uu;
            } else {
              const float sg = fast_sigmoid(gg);
              du[e] = d * gg * sg;
              dg[e] = d * uu * sg * (1.f + gg * (1.f - sg));
            }
          }
          if constexpr (Q != 0) {
            // e5m2 d(gate | up) instead of the bf16 one: bf16-rounded, scaled, two 8-B stores
            const auto qr = rsrc(ep.q8 + (int64_t)m0 * ep.ld_q8, (uint32_t)((int64_t)rows * ep.ld_q8));
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              dg[e] = rbf(dg[e]);
              du[e] = rbf(du[e]);
              qmax = fmaxf(qmax, fmaxf(fabsf(dg[e]), fabsf(du[e])));
            }
            const uint2 og8 = uint2{cvt4<1>(dg[0] * qs, dg[1] * qs, dg[2] * qs, dg[3] * qs),
                                    cvt4<1>(dg[4] * qs, dg[5] * qs, dg[6] * qs, dg[7] * qs)};
            const uint2 ou8 = uint2{cvt4<1>(du[0] * qs, du[1] * qs, du[2] * qs, du[3] * qs),
                                    cvt4<1>(du[4] * qs, du[5] * qs, du[6] * qs, du[7] * qs)};
            const uint32_t cg = ok ? (uint32_t)((int64_t)mr * ep.ld_q8 + f) : 0x80000000u;
            const uint32_t cu = ok ? (uint32_t)((int64_t)mr * ep.ld_q8 + N + f) : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, og8), qr, cg, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, ou8), qr, cu, 0, 0);
            __builtin_amdgcn_sched_barrier(0);  // one step at a time: bounded epilogue registers
          } else {
            const u32x4 og4 = u32x4{pack2(dg[0], dg[1]), pack2(dg[2], dg[3]), pack2(dg[4], dg[5]), pack2(dg[6], dg[7])};
            const u32x4 ou4 = u32x4{pack2(du[0], du[1]), pack2(du[2], du[3]), pack2(du[4], du[5]), pack2(du[6], du[7])};
            if constexpr ((ABL & 256) == 0) {
              // full-line stores as in the plain epilogue: d(gate) rows 0-15 and d(up) rows 16-31 of the
              // wave's 4-KiB LDS staging region; after both column halves, 16 rows x 128 B per output
              char* stg = smem + 2 * BUF_B + w * 4096;
              const int ch = (2 * bp + (q & 1)) * 2 + (q >> 1);
              *reinterpret_cast<u32x4*>(stg + r16 * 128 + ((ch ^ (r16 & 7)) << 4)) = og4;
              *reinterpret_cast<u32x4*>(stg + (16 + r16) * 128 + ((ch ^ (r16 & 7)) << 4)) = ou4;
              if (bp == 1) {
                asm volatile("" ::: "memory");
                const int lc = (lane + z) & 7;
                const int col = n0 + wn * 64 + lc * 8;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                  const int rr = i * 8 + ((lane + z) >> 3);  // staging row: i < 2 gate, else up
                  const u32x4 d = *reinterpret_cast<const u32x4*>(stg + rr * 128 + ((lc ^ (rr & 7)) << 4));
                  const int grow = g * 128 + a * 16 + (rr & 15);
                  const uint32_t off = col < N && (ABL & 8192) == 0
                                           ? (uint32_t)(((int64_t)grow * ldc + (i >= 2 ? N : 0) + col) * 2)
                                           : 0x80000000u;
                  __builtin_amdgcn_raw_buffer_store_b128(d, cr, off, 0, STP);
                }
                asm volatile("" ::: "memory");
              }
            } else {
              const uint32_t cg = ok ? (uint32_t)(((int64_t)mr * ldc + f) * 2) : 0x80000000u;
              const uint32_t cu = ok ? (uint32_t)(((int64_t)mr * ldc + N + f) * 2) : 0x80000000u;
              __builtin_amdgcn_raw_buffer_store_b128(og4, cr, cg, 0, 0);
              __builtin_amdgcn_raw_buffer_store_b128(ou4, cr, cu, 0, 0);
            }
          }
        }
      }
    }
  }

// the q|k|v epilogue per wave: its 64 columns are all q / k (RoPE) or all v (rope_cols % 64 == 0), so a
// wave-uniform branch picks the RoPE body or the plain store body -- the v waves load no tables, whose
// vmcnt waits would also drain the LDS-DMA pieces issued just before them (both bodies store NStores = 16)
template <int EPI, int HD, int ABL, int F8 = 0, int Q = 0, int FORM = 0>
__device__ __forceinline__ void pp_epilogue_any(const f32x4 (&acc)[8][4], bf16_t* __restrict__ C, int M, int N,
                                                int64_t ldc, const PPEpi& ep, int m0, int n0, int g, int wn, int w,
                                                int lane, char* smem, float sc, float qs, float& qmax) {
  if constexpr (EPI == PP_ROPE) {
    static_assert(NStores<PP_ROPE>::v == NStores<PP_STORE>::v, "counted waits assume equal store counts");
    if (n0 + wn * 64 < ep.rope_cols)
      pp_epilogue<PP_ROPE, HD, ABL, F8, Q>(acc, C, M, N, ldc, ep, m0, n0, g, wn, w, lane, smem, sc, qs, qmax);
    else
      pp_epilogue<PP_STORE, HD, ABL, F8, Q>(acc, C, M, N, ldc, ep, m0, n0, g, wn, w, lane, smem, sc, qs, qmax);
  } else {
    pp_epilogue<EPI, HD, ABL, F8, Q, FORM>(acc, C, M, N, ldc, ep, m0, n0, g, wn, w, lane, smem, sc, qs, qmax);
  }
}

// ABL: ablation / A-B builds for profiling only (1-8, 16, 64, 128: wrong results): 1 no LDS-DMA in the
// loop, 2 fragments read only in each tile's first K-tile, 4 no barriers in the loop, 8 no epilogue stores;
// 1024 (correct): every half-tile staged with buffer loads (the default stages full half-tiles with FLAT-global
// LDS loads: bitwise the same, 1.004-1.011x on the fused kernels, profiles/r4_gdma_ab.md)
// F8 (fp8 operands, one 16x16x128 MFMA per 128-deep K-tile of the same 128-B LDS rows): 0 bf16; 1 A e4m3,
// B e4m3 (forward); 2 A e5m2, B e4m3 (input gradient).  A / B are then byte arrays, lda / ldb in bytes.
template <int EPI, int HD, int ABL = 0, int F8 = 0, int Q = 0, int FORM = 0>
__global__ void __launch_bounds__(512, 1) gemm_pp_kernel(const bf16_t* __restrict__ A_, const bf16_t* __restrict__ B_,
                                                         bf16_t* __restrict__ C, int M, int N, int K, int64_t lda,
                                                         int64_t ldb, int64_t ldc, PPEpi ep, int GM) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int ES = F8 ? 1 : 2;       // operand bytes per element
  constexpr int TKE = TK * 2 / ES;     // operand elements per K-tile (128 B per row either way)
  const char* __restrict__ A = reinterpret_cast<const char*>(A_);
  const char* __restrict__ B = reinterpret_cast<const char*>(B_);
  constexpr int NST = NStores<EPI>::v;
  // C stores: non-temporal (aux 2) and, for the plain / RoPE epilogues, full 128-B lines staged
  // through LDS (measured -6 % kernel time together, profiles/r3_gemm_pp.md); ABL 32 / 256 turn
  // them off for A/B
  constexpr int STP = (ABL & 32) ? 0 : 2;
  constexpr int tcols = EPI == PP_SWIGLU ? 128 : TN;  // output columns (units) per tile
  const int tn = (N + tcols - 1) / tcols, tmn = (M + TM - 1) / TM, tiles = tmn * tn;
  const int G = gridDim.x;  // <= tiles (host)
  const int first = xcd_remap(blockIdx.x, G);
  const int my_tiles = (tiles - 1 - first) / G + 1;
  const int nk = K / TKE;
  const int total = my_tiles * nk;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = w >> 2, wn = w & 3;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  const float sc = F8 != 0 ? ep.sa[0] * ep.sb[0] : 1.f;  // fp8 dequantisation of the accumulator
  const float qs = Q != 0 ? ep.qscale[0] : 1.f;           // Q: the fp8 output's scale
  float qmax = 0.f;                                        // Q: running amax of the fp8 output
  int one = 0;  // unit E8M0 block scales of the fp8 MFMA
  if constexpr (F8 != 0) asm volatile("v_mov_b32 %0, 0x7f7f7f7f" : "=v"(one));

  // tile t -> (m0, n0): groups of GM m-panels walked n-major inside the group
  auto coords = [&](int t, int& m0, int& n0) __attribute__((always_inline)) {
    if (GM <= 1) {
      m0 = (t / tn) * TM;
      n0 = (t % tn) * tcols;
    } else {
      const int per = GM * tn, grp = t / per, r = t - grp * per;
      const int gm = (tmn - grp * GM) < GM ? (tmn - grp * GM) : GM;
      m0 = (grp * GM + r % gm) * TM;
      n0 = (r / gm) * tcols;
    }
  };

  // ---- per-lane DMA source offsets (bytes, relative to the half-tile's first row): piece p of this
  // wave = half-tile rows 8 j .. 8 j + 7, j = wn + 4 p; lane -> row 8 j + lane / 8, logical chunk
  // (lane & 7) ^ swizzle(row)
  uint32_t voff[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int hr = 8 * (wn + 4 * p) + (lane >> 3);
    const int lch = (lane & 7) ^ ((hr >> 1) & 7);
    int row = hr;
    if (g == 0 && EPI == PP_SWIGLU) row = ((hr >> 5) & 1) * N + (hr >> 6) * 32 + (hr & 31);  // gate | up rows
    voff[p] = (uint32_t)((int64_t)row * (g == 0 ? ldb : lda) * ES + lch * 16);
  }
  // descriptor of one half-tile of K-tile kt of tile t: A half h (rows m0 + 128 h ..) or B half h
  auto a_rsrc = [&](int m0, int kt, int h) __attribute__((always_inline)) {
    const int64_t e0 = ((int64_t)(m0 + 128 * h) * lda + (int64_t)kt * TKE) * ES;
    const int64_t lim = (int64_t)M * lda * ES - e0;  // bytes to the end of the operand's last row
    return rsrc(A + e0, (uint32_t)(lim > 0 ? (lim < 0x7ffffffe ? lim : 0x7ffffffe) : 0));
  };
  auto b_rsrc = [&](int n0, int kt, int h) __attribute__((always_inline)) {
    const int64_t hrow = EPI == PP_SWIGLU ? 64 * h : 128 * h;  // SwiGLU: half 1 = wave groups 2, 3
    const int64_t e0 = ((int64_t)(n0 + hrow) * ldb + (int64_t)kt * TKE) * ES;
    const int64_t rows = EPI == PP_SWIGLU ? 2 * (int64_t)N : N;
    const int64_t lim = rows * ldb * ES - e0;
    return rsrc(B + e0, (uint32_t)(lim > 0 ? (lim < 0x7ffffffe ? lim : 0x7ffffffe) : 0));
  };
  // stream positions -> (tile, kt): incremental counters
  struct Pos { int lt, kt, m0, n0; };
  auto pos_init = [&](Pos& p, int s) __attribute__((always_inline)) {
    p.lt = s / nk;
    p.kt = s - p.lt * nk;
    coords(first + p.lt * G, p.m0, p.n0);
  };
  auto pos_next = [&](Pos& p) __attribute__((always_inline)) {
    if (++p.kt == nk) {
      p.kt = 0;
      ++p.lt;
      if (p.lt < my_tiles) coords(first + p.lt * G, p.m0, p.n0);
    }
  };
  // group 0: B (both halves) of stream position p -> buffer of p
  auto stage_b = [&](const Pos& p, int s) __attribute__((always_inline)) {
    const uint32_t dst = lds0 + (uint32_t)(s & 1) * BUF_B + 2 * HALF_B + (uint32_t)wn * 1024u;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bool full = EPI == PP_SWIGLU ? p.n0 + 128 <= N : p.n0 + 128 * h + 128 <= N;
      if (!(ABL & 1024) && full) {
        const char* base = B + ((int64_t)(p.n0 + (EPI == PP_SWIGLU ? 64 : 128) * h) * ldb + (int64_t)p.kt * TKE) * ES;
        if constexpr (ND_DMA_BURST) {
          gdma4<4096>(base, voff[0], voff[1], voff[2], voff[3], dst + (uint32_t)h * HALF_B);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) gdma(base, voff[q], dst + (uint32_t)h * HALF_B + (uint32_t)q * 4096u);
        }
      } else {
        const auto r = b_rsrc(p.n0, p.kt, h);
        if constexpr (ND_DMA_BURST) {
          dma4<4096>(r, voff[0], voff[1], voff[2], voff[3], dst + (uint32_t)h * HALF_B);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) dma(r, voff[q], dst + (uint32_t)h * HALF_B + (uint32_t)q * 4096u);
        }
      }
    }
  };
  // group 1: A half h of stream position p
  auto stage_a = [&](const Pos& p, int s, int h) __attribute__((always_inline)) {
    const uint32_t dst = lds0 + (uint32_t)(s & 1) * BUF_B + (uint32_t)h * HALF_B + (uint32_t)wn * 1024u;
    if (!(ABL & 1024) && p.m0 + 128 * h + 128 <= M) {
      const char* base = A + ((int64_t)(p.m0 + 128 * h) * lda + (int64_t)p.kt * TKE) * ES;
      if constexpr (ND_DMA_BURST) {
        gdma4<4096>(base, voff[0], voff[1], voff[2], voff[3], dst);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) gdma(base, voff[q], dst + (uint32_t)q * 4096u);
      }
    } else {
      const auto r = a_rsrc(p.m0, p.kt, h);
      if constexpr (ND_DMA_BURST) {
        dma4<4096>(r, voff[0], voff[1], voff[2], voff[3], dst);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) dma(r, voff[q], dst + (uint32_t)q * 4096u);
      }
    }
  };

  // ---- fragment reads: A rows 16 a + (lane & 15) of half g, B rows (wn & 1) 64 + 16 b + (lane & 15) of
  // half 2 + (wn >> 1); chunk (4 ks + lane / 16) ^ swizzle -- the same per-lane offset for A and B
  const int r16 = lane & 15, q = lane >> 4;
  // bf16: k-step 0 = chunk q, k-step 1 = chunk 4 + q; fp8: the lane's 32 K bytes = chunks 2 q, 2 q + 1
  const int ch0 = F8 ? 2 * q : q, ch1 = F8 ? 2 * q + 1 : 4 + q;
  const uint32_t foff0 = (uint32_t)(r16 * 128 + ((ch0 ^ ((r16 >> 1) & 7)) << 4));
  const uint32_t foff1 = (uint32_t)(r16 * 128 + ((ch1 ^ ((r16 >> 1) & 7)) << 4));
  bf16x8 fa[8][2], fb[4][2];
  auto load_frags = [&](int s) __attribute__((always_inline)) {
    const char* base = smem + (s & 1) * BUF_B;
    const char* ab = base + g * HALF_B;
    const char* bb = base + (2 + (wn >> 1)) * HALF_B + (wn & 1) * 64 * 128;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      fb[b][0] = *reinterpret_cast<const bf16x8*>(bb + b * 2048 + foff0);
      fb[b][1] = *reinterpret_cast<const bf16x8*>(bb + b * 2048 + foff1);
    }
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      fa[a][0] = *reinterpret_cast<const bf16x8*>(ab + a * 2048 + foff0);
      fa[a][1] = *reinterpret_cast<const bf16x8*>(ab + a * 2048 + foff1);
    }
  };

  f32x4 acc[8][4];

  // ---- prologue: K-tile 0 complete plus A0 of K-tile 1, all waves drain, group 1 one barrier behind
  Pos pb, pa1, pa0;  // group 0: B stream; group 1: A1 and A0 streams
  if (g == 0) {
    pos_init(pb, 0);
    stage_b(pb, 0);
    pos_next(pb);  // now K-tile 1
  } else {
    pos_init(pa1, 0);
    stage_a(pa1, 0, 0);  // A0 of K-tile 0 too (A0 runs two K-tiles ahead from then on)
    stage_a(pa1, 0, 1);
    pos_next(pa1);  // K-tile 1
    pos_init(pa0, total > 1 ? 1 : 0);
    if (total > 1) {
      stage_a(pa0, 1, 0);
      pos_next(pa0);  // K-tile 2
    }
  }
  vmwait<0>();
  bar();
  if (g == 1) bar();

  // one K-tile: LOAD(s) + COMPUTE(s).  FIRST (the tile's first K-tile, a separate instantiation so
  // no accumulator PHI merges two definitions): zero accumulator input, and for lt > 0 the previous
  // tile's epilogue inside the LOAD phase
  auto ktile = [&](auto FIRST, int s, int lt, int kt) __attribute__((always_inline)) {
    constexpr bool F = decltype(FIRST)::value;
    const bool fat = F && lt > 0;
    // group 1, the K-tile after a fat phase: the previous tile's stores are younger than A0(s + 1),
    // which this LOAD phase retires -- leave them in flight
    const bool after_fat = !F && kt == 1 && lt > 0;
    const bool more1 = s + 1 < total, more2 = s + 2 < total;
    // ================= LOAD(s)
    auto issue_dma = [&]() __attribute__((always_inline)) {
      if (ABL & 1) {
      } else if (g == 0) {
        if (more1) {
          stage_b(pb, s + 1);
          pos_next(pb);
        }
      } else {
        if (more1) {
          stage_a(pa1, s + 1, 1);
          pos_next(pa1);
        }
        if (more2) {
          stage_a(pa0, s + 2, 0);
          pos_next(pa0);
        }
      }
    };
    // ABL 64: fragment reads ahead of the DMA issue in the plain phases (their latency then runs
    // under the DMA issue); a fat phase keeps DMA -> stores -> reads (the stores must be the youngest)
    bool reads_first = false;
    if constexpr ((ABL & 64) != 0) {
      reads_first = !fat;
      if (reads_first) {
        load_frags(s);
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    issue_dma();
    if (fat) {
      drain();
      if constexpr ((ABL & 8) != 0) {
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) asm volatile("" ::"v"(acc[a][b]));
      } else {
        int m0, n0;
        coords(first + (lt - 1) * G, m0, n0);
        pp_epilogue_any<EPI, HD, ABL, F8, Q, FORM>(acc, C, M, N, ldc, ep, m0, n0, g, wn, w, lane, smem, sc, qs, qmax);
      }
      // the accumulators are free only after the epilogue has read them: keep the fragment reads
      // (96 VGPRs) from being hoisted into it
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    if (!reads_first && (!(ABL & 2) || F)) load_frags(s);
    __builtin_amdgcn_s_waitcnt(LGKM0);
    if (g == 1 && !(ABL & 16))
      vmwait_n<NST>((more1 ? 4 : 0) + (more2 ? 4 : 0) + (fat || after_fat ? NST : 0));  // A0(s + 1) landed
    if (!(ABL & 4)) bar();
    // ================= COMPUTE(s)
    __builtin_amdgcn_s_setprio(1);
    if constexpr (F8 != 0) {
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if constexpr (F) mma8z<F8>(cat16(fb[b][0], fb[b][1]), cat16(fa[a][0], fa[a][1]), acc[a][b], one);
          else mma8<F8>(cat16(fb[b][0], fb[b][1]), cat16(fa[a][0], fa[a][1]), acc[a][b], one);
        }
    } else {
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        if constexpr (F) mma0(fb[b][0], fa[a][0], acc[a][b]);
        else mma(fb[b][0], fa[a][0], acc[a][b]);
      }
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) mma(fb[b][1], fa[a][1], acc[a][b]);
    }
    __builtin_amdgcn_s_setprio(0);
    if (ABL & 16) {
    } else if (g == 0) {
      vmwait_n<NST>(fat ? NST : 0);  // B(s + 1) landed
    } else {
      vmwait_n<NST>((more2 ? 4 : 0) + (fat ? NST : 0));  // A1(s + 1) landed
    }
    if (!(ABL & 4)) bar();
  };
  for (int lt = 0, s = 0; lt < my_tiles; ++lt) {
    ktile(std::true_type{}, s++, lt, 0);
    for (int kt = 1; kt < nk; ++kt) ktile(std::false_type{}, s++, lt, kt);
  }
  drain();
  if constexpr ((ABL & 8) == 0) {
    int m0, n0;
    coords(first + (my_tiles - 1) * G, m0, n0);
    pp_epilogue_any<EPI, HD, ABL, F8, Q, FORM>(acc, C, M, N, ldc, ep, m0, n0, g, wn, w, lane, smem, sc, qs, qmax);
  }
  if (g == 0 && !(ABL & 4)) bar();  // group 1 ran one barrier more
  if constexpr (Q != 0) {  // one amax partial per wave (vector atomic on an ordered-int view)
    qmax = wave_max(qmax);
    if (lane == 0) atomicMax(reinterpret_cast<int*>(ep.qamax + (blockIdx.x * 8 + w) % ep.qparts), __float_as_int(qmax));
  }
}


int g_pp_group_m = [] {
  const char* e = getenv("ND_GEMM_PP_GM");
  return e ? atoi(e) : 4;
}();

int num_cus_pp() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) return 256;
    return v;
  }();
  return n;
}

// A/B builds: nd_gemm_pp_set_variant or ND_GEMM_PP_VARIANT (read once at load).  The product library
// accepts only the correct-result variants (0 default, 32 plain-policy stores, 256 direct stores, 288 both,
// 512 nt SwiGLU-forward stores, 1024 buffer-form pieces, 2048 / 2080 sc1 nt / sc1 stores); the timing-only ablations with wrong results (1-16, 64, 128 and their sums)
// exist only in a -DND_ABLATION build (csrc/build.py --ablation -> _lib/alt/).
bool pp_variant_ok(int v) {
#ifdef ND_ABLATION
  return v >= 0;
#else
  return v == 0 || v == 32 || v == 256 || v == 288 || v == 512 || v == 1024 || v == 2048 || v == 2080;
#endif
}
int g_pp_variant = [] {
  const char* e = getenv("ND_GEMM_PP_VARIANT");
  const int v = e ? atoi(e) : 0;
  return pp_variant_ok(v) ? v : 0;
}();


template <int EPI, int HD, int ABL, int F8 = 0, int Q = 0, int FORM = 0>
int launch_pp_v(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
                const PPEpi& ep, hipStream_t s) {
  const size_t lds = 2 * (size_t)BUF_B + ((ABL & 256) ? 0 : 8 * 4096);  // 128 KiB + 32 KiB C staging
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_pp_kernel<EPI, HD, ABL, F8, Q, FORM>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return (int)attr;
  const int tcols = EPI == PP_SWIGLU ? 128 : TN;
  const int tiles = ((M + TM - 1) / TM) * ((N + tcols - 1) / tcols);
  const int grid = tiles < num_cus_pp() ? tiles : num_cus_pp();
  hipLaunchKernelGGL((gemm_pp_kernel<EPI, HD, ABL, F8, Q, FORM>), dim3(grid), dim3(512), lds, s, (const bf16_t*)A, (const bf16_t*)B,
                     (bf16_t*)C, M, N, K, lda, ldb, ldc, ep, g_pp_group_m);
  ND_LAUNCH_CHECK();
}

template <int EPI, int HD = 64>
int launch_pp(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
              const PPEpi& ep, hipStream_t s) {
  if (g_pp_variant == 1024) return launch_pp_v<EPI, HD, 1024>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
  if constexpr (EPI == PP_SWIGLU)
    if (g_pp_variant == 512) return launch_pp_v<EPI, HD, 512>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);  // nt SwiGLU stores
  if (g_pp_variant == 2048) return launch_pp_v<EPI, HD, 2048>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);  // sc1 nt stores
  if (g_pp_variant == 2080) return launch_pp_v<EPI, HD, 2080>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);  // sc1 stores
#ifdef ND_ABLATION
  if constexpr (EPI == PP_ROPE) {  // epilogue ablations of the q|k|v + RoPE product: 8 none, 16384 no table loads
    if (g_pp_variant == 8) return launch_pp_v<EPI, HD, 8>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    if (g_pp_variant == 16384) return launch_pp_v<EPI, HD, 16384>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    if (g_pp_variant == 8192) return launch_pp_v<EPI, HD, 8192>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
  }
  if constexpr (EPI == PP_DSWIGLU || EPI == PP_SWIGLU) {  // epilogue ablations of the fused MLP products
    if (g_pp_variant == 8) return launch_pp_v<EPI, HD, 8>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    if (g_pp_variant == 4096) return launch_pp_v<EPI, HD, 4096>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    if (g_pp_variant == 8192) return launch_pp_v<EPI, HD, 8192>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
  }
#endif
  if constexpr (EPI == PP_STORE) {
    switch (g_pp_variant) {
#ifdef ND_ABLATION
      case 1: return launch_pp_v<EPI, HD, 1>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
      case 2: return launch_pp_v<EPI, HD, 2>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
      case 3: return launch_pp_v<EPI, HD, 3>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
      case 4: return launch_pp_v<EPI, HD, 4>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
      case 8: return launch_pp_v<EPI, HD, 8>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
      case 15: return launch_pp_v<EPI, HD, 15>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
      case 16: return launch_pp_v<EPI, HD, 16>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
      case 64: return launch_pp_v<EPI, HD, 64>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
      case 128: return launch_pp_v<EPI, HD, 128>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
      case 8192: return launch_pp_v<EPI, HD, 8192>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
#endif
      case 32: return launch_pp_v<EPI, HD, 32>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);    // plain-policy stores
      case 256: return launch_pp_v<EPI, HD, 256>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);  // direct stores
      case 288: return launch_pp_v<EPI, HD, 288>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);  // direct, plain policy
      default: break;
    }
  }
  return launch_pp_v<EPI, HD, 0>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
}

bool pp_shapes_ok(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc) {
  // 16-B pieces and stores; per-lane byte offsets inside one tile stay 32-bit
  return M > 0 && N > 0 && K > 0 && K % TK == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 &&
         lda >= K && ldb >= K && (int64_t)TM * lda * 2 < (1ll << 31) && (int64_t)TN * ldb * 2 < (1ll << 31) &&
         (int64_t)TM * ldc * 2 < (1ll << 31);
}
}  // namespace

// C[M, N] = A[M, K] . B[N, K]^T (bf16, fp32 accumulate).  K % 64 == 0, N % 8 == 0, lda / ldb / ldc % 8
// == 0, 16-B aligned base pointers.
ND_API int nd_gemm_pp(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb,
                      int64_t ldc, hipStream_t s) {
  if (!pp_shapes_ok(M, N, K, lda, ldb, ldc)) return (int)hipErrorInvalidValue;
  PPEpi ep{};
  return launch_pp<PP_STORE>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
}

// q|k|v projection with RoPE on the first rope_cols columns (q and k heads): rows are tokens
// (t = row % T), tables fp32 [T, hd], hd in {32, 64}, rope_cols % 64 == 0.
ND_API int nd_gemm_pp_rope(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb,
                           int64_t ldc, const float* cosT, const float* sinT, int T, int hd, int rope_cols,
                           hipStream_t s) {
  if (!pp_shapes_ok(M, N, K, lda, ldb, ldc) || (hd != 32 && hd != 64) || rope_cols % 64 || T <= 0)
    return (int)hipErrorInvalidValue;
  PPEpi ep{};
  ep.cosT = cosT; ep.sinT = sinT; ep.T = T; ep.rope_cols = rope_cols;
  return hd == 64 ? launch_pp<PP_ROPE, 64>(A, B, C, M, N, K, lda, ldb, ldc, ep, s)
                  : launch_pp<PP_ROPE, 32>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
}

// The SwiGLU pair's saved-tensor form (FORM of pp_epilogue): 0 gate / up, 1 the coefficient form.  ONE switch for
// the forward and backward launchers of every dtype, so the two sides of a step always agree; ND_MLP_COEF at load,
// nd_mlp_coef_set for A/B (set it only between steps: a forward saved in one form must be read back in it).
int g_mlp_coef = [] {
  const char* e = getenv("ND_MLP_COEF");
  return e ? (atoi(e) != 0) : ND_MLP_COEF_DEFAULT;
}();
template <int EPI, int F8 = 0, int Q = 0>
int launch_mlp(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
               const PPEpi& ep, hipStream_t s) {
  if (g_mlp_coef) {
    if constexpr (F8 == 0) {  // the store-policy A/B variants (bf16 only)
      if (EPI == PP_SWIGLU && g_pp_variant == 512)
        return launch_pp_v<PP_SWIGLU, 64, 512, 0, 0, 1>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
      if (g_pp_variant == 2048) return launch_pp_v<EPI, 64, 2048, 0, 0, 1>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
      if (g_pp_variant == 2080) return launch_pp_v<EPI, 64, 2080, 0, 0, 1>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    }
    return launch_pp_v<EPI, 64, 0, F8, Q, 1>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
  }
  if constexpr (F8 == 0) return launch_pp<EPI>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);  // incl. the A/B variants
  else return launch_pp_v<EPI, 64, 0, F8, Q>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
}

// gate|up projection + SwiGLU: B = fused weight [2F, K] (gate rows then up rows), gu = C [M, 2F]
// (ldc), act [M, F] (ld_act).  F % 8 == 0.
ND_API int nd_gemm_pp_swiglu(const void* A, const void* B, void* gu, void* act, int M, int F, int K, int64_t lda,
                             int64_t ldb, int64_t ldc, int64_t ld_act, hipStream_t s) {
  if (!pp_shapes_ok(M, F, K, lda, ldb, ldc) || ldc < 2 * (int64_t)F || ld_act % 8 || ld_act < F ||
      (int64_t)2 * F * ldb * 2 >= (1ll << 31) || (int64_t)TM * ld_act * 2 >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  PPEpi ep{};
  ep.act = (bf16_t*)act; ep.ld_act = ld_act;
  return launch_mlp<PP_SWIGLU>(A, B, gu, M, F, K, lda, ldb, ldc, ep, s);
}

// down-projection input gradient fused with the SwiGLU backward: d(act) = A . B^T (A = dY [M, K],
// B = W_down^T [F, K]) is never stored; reads gu [M, 2F] and writes dgu [M, 2F].
ND_API int nd_gemm_pp_dswiglu(const void* A, const void* B, const void* gu, void* dgu, int M, int F, int K,
                              int64_t lda, int64_t ldb, int64_t ld_gu, int64_t ld_dgu, hipStream_t s) {
  if (!pp_shapes_ok(M, F, K, lda, ldb, ld_dgu) || ld_gu % 8 || ld_gu < 2 * (int64_t)F || ld_dgu < 2 * (int64_t)F ||
      (int64_t)TM * ld_gu * 2 >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  PPEpi ep{};
  ep.gu = (const bf16_t*)gu; ep.ld_gu = ld_gu;
  return launch_mlp<PP_DSWIGLU>(A, B, dgu, M, F, K, lda, ldb, ld_dgu, ep, s);
}

// ---- fp8 operands (A, B byte arrays, lda / ldb in bytes = elements): C = bf16(sa sb A . B^T) and the same
// fused epilogues on the dequantised accumulator.  fa: A's format (0 e4m3, 1 e5m2); B is e4m3.  K % 128 == 0.
namespace {
bool pp_f8_ok(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int fa, const float* sa, const float* sb) {
  return M > 0 && N > 0 && K > 0 && K % 128 == 0 && N % 8 == 0 && lda % 16 == 0 && ldb % 16 == 0 && ldc % 8 == 0 &&
         lda >= K && ldb >= K && (int64_t)TM * lda < (1ll << 31) && (int64_t)TN * ldb < (1ll << 31) &&
         (int64_t)TM * ldc * 2 < (1ll << 31) && (fa == 0 || fa == 1) && sa && sb;
}
template <int EPI, int HD = 64>
int launch_pp8(int fa, const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
               const PPEpi& ep, hipStream_t s) {
  return fa == 0 ? launch_pp_v<EPI, HD, 0, 1>(A, B, C, M, N, K, lda, ldb, ldc, ep, s)
                 : launch_pp_v<EPI, HD, 0, 2>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
}
}  // namespace

ND_API int nd_gemm_pp_f8(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb,
                         int64_t ldc, const float* sa, const float* sb, int fa, hipStream_t s) {
  if (!pp_f8_ok(M, N, K, lda, ldb, ldc, fa, sa, sb)) return (int)hipErrorInvalidValue;
  PPEpi ep{};
  ep.sa = sa; ep.sb = sb;
  return launch_pp8<PP_STORE>(fa, A, B, C, M, N, K, lda, ldb, ldc, ep, s);
}

ND_API int nd_gemm_pp_rope_f8(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb,
                              int64_t ldc, const float* sa, const float* sb, const float* cosT, const float* sinT, int T,
                              int hd, int rope_cols, hipStream_t s) {
  if (!pp_f8_ok(M, N, K, lda, ldb, ldc, 0, sa, sb) || (hd != 32 && hd != 64) || rope_cols % 64 || T <= 0)
    return (int)hipErrorInvalidValue;
  PPEpi ep{};
  ep.cosT = cosT; ep.sinT = sinT; ep.T = T; ep.rope_cols = rope_cols; ep.sa = sa; ep.sb = sb;
  return hd == 64 ? launch_pp_v<PP_ROPE, 64, 0, 1>(A, B, C, M, N, K, lda, ldb, ldc, ep, s)
                  : launch_pp_v<PP_ROPE, 32, 0, 1>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
}

ND_API int nd_gemm_pp_swiglu_f8(const void* A, const void* B, void* gu, void* act, int M, int F, int K, int64_t lda,
                                int64_t ldb, int64_t ldc, int64_t ld_act, const float* sa, const float* sb,
                                hipStream_t s) {
  if (!pp_f8_ok(M, F, K, lda, ldb, ldc, 0, sa, sb) || ldc < 2 * (int64_t)F || ld_act % 8 || ld_act < F ||
      (int64_t)2 * F * ldb >= (1ll << 31) || (int64_t)TM * ld_act * 2 >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  PPEpi ep{};
  ep.act = (bf16_t*)act; ep.ld_act = ld_act; ep.sa = sa; ep.sb = sb;
  return launch_mlp<PP_SWIGLU, 1>(A, B, gu, M, F, K, lda, ldb, ldc, ep, s);
}

// A = dY in e5m2 (fa = 1) or e4m3 (fa = 0)
ND_API int nd_gemm_pp_dswiglu_f8(const void* A, const void* B, const void* gu, void* dgu, int M, int F, int K,
                                 int64_t lda, int64_t ldb, int64_t ld_gu, int64_t ld_dgu, const float* sa,
                                 const float* sb, int fa, hipStream_t s) {
  if (!pp_f8_ok(M, F, K, lda, ldb, ld_dgu, fa, sa, sb) || ld_gu % 8 || ld_gu < 2 * (int64_t)F ||
      ld_dgu < 2 * (int64_t)F || (int64_t)TM * ld_gu * 2 >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  PPEpi ep{};
  ep.gu = (const bf16_t*)gu; ep.ld_gu = ld_gu; ep.sa = sa; ep.sb = sb;
  return fa == 0 ? launch_mlp<PP_DSWIGLU, 1>(A, B, dgu, M, F, K, lda, ldb, ld_dgu, ep, s)
                 : launch_mlp<PP_DSWIGLU, 2>(A, B, dgu, M, F, K, lda, ldb, ld_dgu, ep, s);
}

// Q forms: the SwiGLU output as e4m3 act8 [M, F] (ld_q8) INSTEAD of the bf16 act / the d(gate|up) as e5m2
// dgu8 [M, 2F] INSTEAD of the bf16 dgu, with the delayed-scaling scale `qscale` and amax into `qparts`
// partial slots -- bitwise a separate nd_fp8_cast of the bf16 tensor the plain form writes.
ND_API int nd_gemm_pp_swiglu_f8q(const void* A, const void* B, void* gu, void* act8, int M, int F, int K, int64_t lda,
                                 int64_t ldb, int64_t ldc, int64_t ld_q8, const float* sa, const float* sb,
                                 const float* qscale, float* qamax, int qparts, hipStream_t s) {
  if (!pp_f8_ok(M, F, K, lda, ldb, ldc, 0, sa, sb) || ldc < 2 * (int64_t)F || ld_q8 % 8 || ld_q8 < F || !qscale ||
      !qamax || qparts < 1 || (int64_t)2 * F * ldb >= (1ll << 31) || (int64_t)TM * ld_q8 >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  PPEpi ep{};
  ep.sa = sa; ep.sb = sb; ep.q8 = (uint8_t*)act8; ep.ld_q8 = ld_q8; ep.qscale = qscale; ep.qamax = qamax;
  ep.qparts = qparts;
  return launch_mlp<PP_SWIGLU, 1, 1>(A, B, gu, M, F, K, lda, ldb, ldc, ep, s);
}

ND_API int nd_gemm_pp_dswiglu_f8q(const void* A, const void* B, const void* gu, void* dgu8, int M, int F, int K,
                                  int64_t lda, int64_t ldb, int64_t ld_gu, int64_t ld_q8, const float* sa,
                                  const float* sb, int fa, const float* qscale, float* qamax, int qparts,
                                  hipStream_t s) {
  if (!pp_f8_ok(M, F, K, lda, ldb, 2 * (int64_t)F, fa, sa, sb) || ld_gu % 8 || ld_gu < 2 * (int64_t)F ||
      ld_q8 % 8 || ld_q8 < 2 * (int64_t)F || !qscale || !qamax || qparts < 1 || (int64_t)TM * ld_gu * 2 >= (1ll << 31) ||
      (int64_t)TM * ld_q8 >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  PPEpi ep{};
  ep.gu = (const bf16_t*)gu; ep.ld_gu = ld_gu; ep.sa = sa; ep.sb = sb; ep.q8 = (uint8_t*)dgu8; ep.ld_q8 = ld_q8;
  ep.qscale = qscale; ep.qamax = qamax; ep.qparts = qparts;
  // C (the bf16 dgu) is not written: the Q epilogue stores through ep.q8 only
  return fa == 0 ? launch_mlp<PP_DSWIGLU, 1, 1>(A, B, dgu8, M, F, K, lda, ldb, 2 * (int64_t)F, ep, s)
                 : launch_mlp<PP_DSWIGLU, 2, 1>(A, B, dgu8, M, F, K, lda, ldb, 2 * (int64_t)F, ep, s);
}

// returns the previous variant, or -1 (nothing changed) for a variant this build does not contain
ND_API int nd_gemm_pp_set_variant(int v) {
  if (!pp_variant_ok(v)) return -1;
  const int old = g_pp_variant;
  g_pp_variant = v;
  return old;
}

// the SwiGLU saved-tensor form (see g_mlp_coef); v < 0 only reads it.  Returns the previous setting.
ND_API int nd_mlp_coef_set(int v) {
  const int old = g_mlp_coef;
  if (v >= 0) g_mlp_coef = v != 0;
  return old;
}

ND_API int nd_gemm_pp_set_group_m(int gm) {
  const int old = g_pp_group_m;
  if (gm >= 0) g_pp_group_m = gm;
  return old;
}
