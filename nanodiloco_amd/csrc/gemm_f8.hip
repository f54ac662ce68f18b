// fp8 x fp8 -> bf16 projection GEMM for gfx950 (the --fp8 recipe's forward e4m3 x e4m3 and input-gradient
// e5m2 x e4m3 GEMMs; `--fp8-gemm hip`, ops/fp8.py):  C[M, N] = bf16(sa * sb * A[M, K] . B[N, K]^T).
//
// Persistent 4-wave workgroups (one per CU), 256 x 256 tiles, each wave a 128 x 128 quadrant of
// v_mfma_scale_f32_32x32x64_f8f6f4 accumulators (256 AGPRs), operands streamed through a padded LDS
// block layout by LDS-DMA (or VGPR-staged loads for long K, LDM 2), C staged through LDS into full-line
// stores.  The bf16 projection GEMMs with fused epilogues live in csrc/gemm_pp.hip (two waves per SIMD in
// opposite load / MFMA phases); the round-1 / round-2 bf16 kernels this file used to hold were
// superseded by it and removed (profiles/r2_gemm_ab.md, profiles/r3_gemm_pp.md).
#include "common.h"
#include <cstdlib>
#include <type_traits>

using namespace nd;

namespace {
constexpr int TM = 256, TN = 256, TK = 64;

// s_waitcnt immediate (gfx9 encoding) for lgkmcnt(0) with vmcnt / expcnt at their maxima
constexpr int LGKM0 = 0xC07F;

// one LDS-DMA wave-instruction: 64 lanes x 16 B from sbase + voff (per lane) to LDS [lds, lds + 1 KiB)
__device__ __forceinline__ void glds(const void* sbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_n(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7FFFFFFF, 0x00020000);
}

// SWZ 2: padded block layout.  A half-tile is 16 LDS blocks of 1056 B (8 rows x 128 B + 32 B pad);
// block b holds rows b, b + 16, ..., b + 112 unswizzled, so every LDS-DMA lane octet reads one whole
// 128-B row in ascending order (one cache access per line), and a ds_read_b128 lane group (16 rows
// 16 apart in block index) lands on 16 distinct 16-B bank slots thanks to the 32-B pad.
constexpr int BLOCK_P = 1056;                 // bytes per padded block
constexpr int HALF_P = 16 * BLOCK_P / 2;      // elements per padded half-tile

// ---------------------------------------------------------------------------------------------
// fp8 x fp8 -> bf16 projection GEMM (the --fp8 recipe's forward e4m3 x e4m3 and input-gradient
// e5m2 x e4m3 GEMMs; replaces torch._scaled_mm).  C = bf16(sa * sb * A . B^T), sa / sb device scalars
// (the recipe's inverse scales: delayed scaling, no host sync).
//
// A K-tile of 128 fp8 = 128 B per row is byte-for-byte the bf16 kernel's 64-element K-tile, so the
// LDS image, the LDS-DMA staging stream (persistent grid, padded block layout) and the C epilogue
// path are those of the round-2 bf16 4-wave kernel (padded block layout); operands addressed as bf16 pairs.
// The matrix op is v_mfma_scale_f32_32x32x64_f8f6f4 (unit block scales, E8M0 127): twice the
// cycles of the bf16 32x32x16 at four times the K, i.e. 2x the bf16 rate.  Per wave 128 x 128 =
// 4 x 4 accumulators of 32 x 32 (256 AGPRs); a 64-B k-step needs 4 + 4 fragments of 32 B per
// lane (lane l: row l % 32, bytes (l / 32) * 32 + [0, 32) of the step -- A and B use the same
// byte -> k assignment, so the MFMA's internal K order does not matter), double-buffered exactly
// like the bf16 kernel's two k-steps.  Accumulator lane l holds token row l % 32 and output
// columns 8 i + 4 (l / 32) + [0, 4) of its 32-column block (i = 0..3).
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4v __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ i32x8 frag8(const bf16_t* half, int row, int kc) {
  const bf16_t* p = &half[(row & 15) * (BLOCK_P / 2) + (row >> 4) * 64 + kc];
  const i32x4v lo = *reinterpret_cast<const i32x4v*>(p);
  const i32x4v hi = *reinterpret_cast<const i32x4v*>(p + 8);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// D += A . B^T with A / B fp8 (CB = format of the first operand, BL = of the second: 0 e4m3,
// 1 e5m2), unit E8M0 scales (`one` = 0x7F7F7F7F), accumulator pinned to AGPRs as in mfma16a
template <int CB, int BL>
__device__ __forceinline__ void mfma32f8(const i32x8& a, const i32x8& b, f32x16& c, int one) {
  if constexpr (CB == 0 && BL == 0)
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]" : "+a"(c) : "v"(a), "v"(b), "v"(one));
  else if constexpr (CB == 0 && BL == 1)
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0] blgp:1" : "+a"(c) : "v"(a), "v"(b), "v"(one));
  else if constexpr (CB == 1 && BL == 0)
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0] cbsz:1" : "+a"(c) : "v"(a), "v"(b), "v"(one));
  else
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0] cbsz:1 blgp:1" : "+a"(c) : "v"(a), "v"(b), "v"(one));
}

// 16-B buffer load the compiler does not track (LDM 3): the caller waits with an explicit vmcnt
__device__ __forceinline__ u32x4 bload_untracked(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  u32x4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r) : "memory");
  return v;
}

// the same with a zero accumulator input (first k-step of a tile): no per-tile AGPR zeroing
template <int CB, int BL>
__device__ __forceinline__ void mfma32f8z(const i32x8& a, const i32x8& b, f32x16& c, int one) {
  if constexpr (CB == 0 && BL == 0)
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, 0, %3, %3 op_sel_hi:[0,0,0]" : "=a"(c) : "v"(a), "v"(b), "v"(one));
  else if constexpr (CB == 0 && BL == 1)
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, 0, %3, %3 op_sel_hi:[0,0,0] blgp:1" : "=a"(c) : "v"(a), "v"(b), "v"(one));
  else if constexpr (CB == 1 && BL == 0)
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, 0, %3, %3 op_sel_hi:[0,0,0] cbsz:1" : "=a"(c) : "v"(a), "v"(b), "v"(one));
  else
    asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, 0, %3, %3 op_sel_hi:[0,0,0] cbsz:1 blgp:1" : "=a"(c) : "v"(a), "v"(b), "v"(one));
}

// FA / FB: formats of A (tokens) and B (weight); M, N in rows, K / lda / ldb in bf16 PAIRS (fp8 / 2)
// LDM: 0 = LDS-DMA pieces ahead of each k-step-1 MFMA group, 1 = one DMA piece after each MFMA,
// 2 = VGPR staging (buffer_load_dwordx4 one K-tile ahead into 64 VGPRs, ds_write_b128 between the
// k-step-1 MFMAs, the next K-tile's loads issued right behind the writes)
template <int FA, int FB, int LDM>
__global__ void __launch_bounds__(256, 1) gemm4_f8_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                          bf16_t* __restrict__ C, int M, int N, int K, int64_t lda,
                                                          int64_t ldb, int64_t ldc, const float* __restrict__ sa,
                                                          const float* __restrict__ sb, int GM) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  constexpr int HS = HALF_P, BS = 4 * HS;
  const int tn = (N + TN - 1) / TN, tmn = (M + TM - 1) / TM, tiles = tmn * tn;
  const int G = gridDim.x;
  const int first = xcd_remap(blockIdx.x, G);
  const int my_tiles = first < tiles ? (tiles - 1 - first) / G + 1 : 0;
  const int nk = K / TK;
  const int total = my_tiles * nk;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int wr = __builtin_amdgcn_readfirstlane(w);
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf16_t*)smem);
  const float scale = sa[0] * sb[0];

  int s_tile = first, s_kt = 0;
  auto coords = [&](int t, int& m0, int& n0) __attribute__((always_inline)) {
    if (GM <= 1) {
      m0 = (t / tn) * TM;
      n0 = (t % tn) * TN;
    } else {
      const int per = GM * tn, grp = t / per, r = t - grp * per;
      const int gm = (tmn - grp * GM) < GM ? (tmn - grp * GM) : GM;
      m0 = (grp * GM + r % gm) * TM;
      n0 = (r / gm) * TN;
    }
  };
  int s_m0, s_n0;
  coords(s_tile, s_m0, s_n0);
  uint32_t va[2][4], vb[2][4];
  auto offsets = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int hr = (w + 4 * p) + 16 * (lane >> 3), lch = lane & 7, r = 128 * h + hr;
        int ar = s_m0 + r;
        ar = (ar < M ? ar : M - 1) - s_m0;
        va[h][p] = (uint32_t)(((int64_t)ar * lda + lch * 8) * 2);
        int br = s_n0 + r;
        br = (br < N ? br : N - 1) - s_n0;
        vb[h][p] = (uint32_t)(((int64_t)br * ldb + lch * 8) * 2);
      }
  };
  offsets();
  auto stage_piece = [&](int buf, int j) __attribute__((always_inline)) {
    const uint32_t dst = lds0 + (uint32_t)(buf * BS * 2);
    const int h = (j >> 2) & 1, p = j & 3;
    if (j < 8)
      glds(A + (int64_t)s_m0 * lda + (int64_t)s_kt * TK, va[h][p], dst + (uint32_t)((h * HS) * 2 + (wr + 4 * p) * BLOCK_P));
    else
      glds(B + (int64_t)s_n0 * ldb + (int64_t)s_kt * TK, vb[h][p], dst + (uint32_t)(((2 + h) * HS) * 2 + (wr + 4 * p) * BLOCK_P));
  };
  auto advance = [&]() __attribute__((always_inline)) {
    if (++s_kt == nk) {
      s_kt = 0;
      s_tile += G;
      if (s_tile < tiles) {
        coords(s_tile, s_m0, s_n0);
        offsets();
      }
    }
  };
  auto stage_next = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 16; ++j) stage_piece(buf, j);
    advance();
  };
  // LDM 2: piece j of the stream's current K-tile -> VGPRs, and VGPRs -> LDS (the DMA's lane-linear image)
  auto load_piece = [&](int j) __attribute__((always_inline)) -> u32x4 {
    const int h = (j >> 2) & 1, p = j & 3;
    if constexpr (LDM == 3) {
      if (j < 8) return bload_untracked(make_rsrc(A + (int64_t)s_m0 * lda + (int64_t)s_kt * TK), va[h][p]);
      return bload_untracked(make_rsrc(B + (int64_t)s_n0 * ldb + (int64_t)s_kt * TK), vb[h][p]);
    }
    if (j < 8) return __builtin_amdgcn_raw_buffer_load_b128(make_rsrc(A + (int64_t)s_m0 * lda + (int64_t)s_kt * TK), va[h][p], 0, 0);
    return __builtin_amdgcn_raw_buffer_load_b128(make_rsrc(B + (int64_t)s_n0 * ldb + (int64_t)s_kt * TK), vb[h][p], 0, 0);
  };
  auto write_piece = [&](int buf, int j, const u32x4& v) __attribute__((always_inline)) {
    const int h = (j >> 2) & 1, p = j & 3;
    char* d = reinterpret_cast<char*>(smem) + buf * BS * 2 + (j < 8 ? h : 2 + h) * HS * 2 + (w + 4 * p) * BLOCK_P + lane * 16;
    *reinterpret_cast<u32x4*>(d) = v;
  };
  u32x4 stg[16];
  auto ord = [](int k) __attribute__((always_inline)) { return (k & 1) * 8 + (k >> 1); };  // k-step-1 piece order

  f32x16 acc[4][4];  // written first by mfma32f8z
  if (total == 0) return;
  const int one = 0x7F7F7F7F;

  if constexpr (LDM >= 2) {
    // pieces in the k-step-1 loop's order (0, 8, 1, 9, ...): the compiler's vmcnt bookkeeping
    // then sees the same issue order on every path into the loop and can count exactly
#pragma unroll
    for (int k = 0; k < 16; ++k) stg[ord(k)] = load_piece(ord(k));
    advance();
    if constexpr (LDM == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < 16; ++k) write_piece(0, ord(k), stg[ord(k)]);
    if (total > 1) {
#pragma unroll
      for (int k = 0; k < 16; ++k) stg[ord(k)] = load_piece(ord(k));
      advance();
      if constexpr (LDM == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int k = 0; k < 16; ++k) write_piece(1, ord(k), stg[ord(k)]);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) stg[ord(k)] = load_piece(ord(k));
    advance();
    __builtin_amdgcn_s_waitcnt(LGKM0);
  } else {
  stage_next(0);
  if (total > 1) {
    stage_next(1);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  const int r32 = lane & 31, kb = (lane >> 5) * 16;  // kb: element (bf16-pair) offset in a 64-B k-step
  i32x8 fa0[4], fb0[4], fa1[4], fb1[4];
  {
    const bf16_t* at = smem + wm * HS;
    const bf16_t* bt = smem + (2 + wn) * HS;
#pragma unroll
    for (int b = 0; b < 4; ++b) fb0[b] = frag8(bt, b * 32 + r32, kb);
#pragma unroll
    for (int a = 0; a < 4; ++a) fa0[a] = frag8(at, a * 32 + r32, kb);
  }
  for (int lt = 0; lt < my_tiles; ++lt) {
    for (int kt = 0; kt < nk; ++kt) {
      const int g = lt * nk + kt;
      const int buf = g & 1;
      const bool more1 = g + 1 < total, more2 = g + 2 < total;
      const bf16_t* at = smem + buf * BS + wm * HS;
      const bf16_t* bt = smem + buf * BS + (2 + wn) * HS;
      __builtin_amdgcn_s_waitcnt(LGKM0);
      if (kt == 0) {  // first k-step of a tile: the MFMAs start from a zero accumulator
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          fb1[a] = frag8(bt, a * 32 + r32, 32 + kb);
          fa1[a] = frag8(at, a * 32 + r32, 32 + kb);
#pragma unroll
          for (int b = 0; b < 4; ++b) mfma32f8z<FB, FA>(fb0[b], fa0[a], acc[a][b], one);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          fb1[a] = frag8(bt, a * 32 + r32, 32 + kb);
          fa1[a] = frag8(at, a * 32 + r32, 32 + kb);
#pragma unroll
          for (int b = 0; b < 4; ++b) mfma32f8<FB, FA>(fb0[b], fa0[a], acc[a][b], one);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (more1 && LDM < 2) {
        if (kt == 0 && lt > 0) {
          asm volatile("s_waitcnt vmcnt(32)" ::: "memory");  // K-tile g + 1 was issued before the 32 stores
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      __builtin_amdgcn_s_waitcnt(LGKM0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const bf16_t* an = smem + (buf ^ 1) * BS + wm * HS;
      const bf16_t* bn = smem + (buf ^ 1) * BS + (2 + wn) * HS;
      const bool stage_now = more2;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        if constexpr (LDM >= 2) {
          // VGPR staging: K-tile g + 2 (loaded one K-tile ago) into the released buffer, and the
          // same piece of K-tile g + 3 loaded right behind it
          fb0[a] = frag8(bn, a * 32 + r32, kb);
          fa0[a] = frag8(an, a * 32 + r32, kb);
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            mfma32f8<FB, FA>(fb1[b], fa1[a], acc[a][b], one);
            // unconditional (past the stream's end: rewrites a finished tile's pieces into a buffer
            // nobody reads), so every path has the same VMEM issue order and hipcc's vmcnt waits
            // stay exact (a conditional load made it drain to vmcnt(0) every K-tile)
            const int j = (b & 1) * 8 + 2 * a + (b >> 1);
            if constexpr (LDM == 3) {
              // untracked loads: each piece's load is the 16th-newest VMEM op (plus the tile's 32
              // stores right after an epilogue, which stay in flight)
              if (kt == 0 && lt > 0) asm volatile("s_waitcnt vmcnt(47)" ::: "memory");
              else asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
            }
            write_piece(buf, j, stg[j]);
            stg[j] = load_piece(j);
          }
        } else if constexpr (LDM == 1) {
          // one LDS-DMA piece after each MFMA: a piece's issue stall overlaps the MFMA before it
          fb0[a] = frag8(bn, a * 32 + r32, kb);  // past the stream's end: reads unused LDS
          fa0[a] = frag8(an, a * 32 + r32, kb);
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            mfma32f8<FB, FA>(fb1[b], fa1[a], acc[a][b], one);
            if (stage_now) stage_piece(buf, (b & 1) * 8 + 2 * a + (b >> 1));
          }
        } else {
          if (stage_now) {
            stage_piece(buf, 2 * a);
            stage_piece(buf, 2 * a + 1);
            stage_piece(buf, 8 + 2 * a);
            stage_piece(buf, 9 + 2 * a);
          }
          fb0[a] = frag8(bn, a * 32 + r32, kb);  // past the stream's end: reads unused LDS
          fa0[a] = frag8(an, a * 32 + r32, kb);
#pragma unroll
          for (int b = 0; b < 4; ++b) mfma32f8<FB, FA>(fb1[b], fa1[a], acc[a][b], one);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (LDM >= 2 || stage_now) advance();
    }
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 7" ::: "memory");  // 16-pass MFMA results -> VALU
    const int c_tile = first + lt * G;
    int m0, n0;
    coords(c_tile, m0, n0);
    // C through the wave's own LDS staging region (behind the K-tile buffers), in fp32: per pass
    // 16 rows x 64 columns of two accumulator blocks (the lanes holding those rows write 16-B
    // pieces straight from the accumulators), then 8 lanes per row read 8 columns back, apply the
    // scale, round once to bf16 and store whole 128-B lines; every wave issues exactly 32 stores.
    // (Scaling in registers before the staging made hipcc keep accumulators in VGPRs and spill.)
    const __amdgpu_buffer_rsrc_t crs = make_rsrc_n(C + (int64_t)m0 * ldc, (uint32_t)((int64_t)(M - m0 < TM ? M - m0 : TM) * ldc * 2));
    constexpr int RSF = 68;  // fp32 staging row stride (floats): 256 B + 16 B pad
    float* cst = reinterpret_cast<float*>(smem + 2 * BS) + w * (16 * RSF);
    const int q8 = lane >> 3;
#pragma unroll
    for (int pass = 0; pass < 16; ++pass) {
      const int a = pass >> 2, bh = ((pass >> 1) & 1) * 2, hh = pass & 1;  // rows hh * 16 + [0, 16)
      if (((lane >> 4) & 1) == hh) {
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const f32x16& v = acc[a][bh + bb];
            const int col = bb * 32 + i * 8 + (lane >> 5) * 4;
            *reinterpret_cast<f32x4*>(cst + (lane & 15) * RSF + col) = f32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]};
          }
      }
      // lanes read what other lanes wrote: keep hipcc from reordering the LDS accesses across
      // (the hardware runs one wave's LDS instructions in order)
      asm volatile("" ::: "memory");
      const int ccol = n0 + wn * 128 + bh * 32 + (lane & 7) * 8;
      const uint32_t coff = ccol < N ? (uint32_t)(ccol * 2) : 0x80000000u;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = i * 8 + q8;
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(cst + row * RSF + (lane & 7) * 8);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(cst + row * RSF + (lane & 7) * 8 + 4);
        const u32x4 d = u32x4{pack2(x0[0] * scale, x0[1] * scale), pack2(x0[2] * scale, x0[3] * scale),
                              pack2(x1[0] * scale, x1[1] * scale), pack2(x1[2] * scale, x1[3] * scale)};
        const int mr = wm * 128 + a * 32 + hh * 16 + row;
        __builtin_amdgcn_raw_buffer_store_b128(d, crs, coff == 0x80000000u ? coff : coff + (uint32_t)(mr * ldc * 2), 0, 2);
      }
      asm volatile("" ::: "memory");
    }
  }
}

// Variants (ND_GEMM_VARIANT or nd_gemm_set_variant, for in-process A/B): 0 = 8 waves, four barrier-
// separated phases per K-tile; 1 = 8 waves, register-pipelined, one barrier per K-tile; 2 = 4 waves of
// 128 x 128 (one wave per SIMD); 3 = variant 2 as a persistent grid with a cross-tile DMA stream;
// 4 = variant 3 with the half-swap LDS swizzle (coalesced 64-B DMA source quads); 5 = variant 3 with
// the padded block layout (whole ascending 128-B rows per DMA lane octet, conflict-free reads);
// 6 = variant 5 with buffer_load ... lds DMA; 7 = variant 5 on a plain (one tile per workgroup)
// grid; 8 = 5; 9 = 5 with plain C stores; 10 (default) = variant 5 with each k-step-1 DMA piece issued
// between MFMAs (+1.8 % over 5).  Measured against hipBLASLt on the Llama-150M shapes: docs/DESIGN.md.
int g_group_m = [] {
  const char* e = getenv("ND_GEMM_GROUP_M");
  return e ? atoi(e) : 4;
}();

int num_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    return v;
  }();
  return n;
}

int g_f8_variant = [] {
  const char* e = getenv("ND_GEMM_F8_VARIANT");
  return e ? atoi(e) : -1;  // -1: auto (see launch_f8)
}();

template <int FA, int FB, int LDM>
int launch_f8_v(const void* A, const void* B, void* C, int M, int N, int K2, int64_t lda2, int64_t ldb2, int64_t ldc,
              const float* sa, const float* sb, hipStream_t s) {
  const size_t lds = 2 * (size_t)(4 * HALF_P) * sizeof(bf16_t) + 4 * 16 * 68 * sizeof(float);  // 149 KiB
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm4_f8_kernel<FA, FB, LDM>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return (int)attr;
  const int tiles = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  const int grid = tiles < num_cus() ? tiles : num_cus();
  hipLaunchKernelGGL((gemm4_f8_kernel<FA, FB, LDM>), dim3(grid), dim3(256), lds, s, (const bf16_t*)A, (const bf16_t*)B,
                     (bf16_t*)C, M, N, K2, lda2, ldb2, ldc, sa, sb, g_group_m);
  ND_LAUNCH_CHECK();
}
// ND_GEMM_F8_VARIANT / nd_gemm_set_f8_variant: -1 (default) = auto by K, 1 = one DMA piece per MFMA
// in k-step 1, 0 = four pieces ahead of each group of four MFMAs, 2 = VGPR-staged loads
template <int FA, int FB>
int launch_f8(const void* A, const void* B, void* C, int M, int N, int K2, int64_t lda2, int64_t ldb2, int64_t ldc,
              const float* sa, const float* sb, hipStream_t s) {
  // auto: VGPR staging for long reductions (K > 4096 fp8: 0.81x vs 0.74x hipBLASLt at K = 5376), the
  // interleaved DMA otherwise (its prologue and post-epilogue waits are shorter; profiles/r2_fp8_gemm_ab.md)
  const int v = g_f8_variant >= 0 ? g_f8_variant : (K2 > 2048 ? 2 : 1);
  if (v == 2) return launch_f8_v<FA, FB, 2>(A, B, C, M, N, K2, lda2, ldb2, ldc, sa, sb, s);
  if (v == 3) return launch_f8_v<FA, FB, 3>(A, B, C, M, N, K2, lda2, ldb2, ldc, sa, sb, s);
  return v ? launch_f8_v<FA, FB, 1>(A, B, C, M, N, K2, lda2, ldb2, ldc, sa, sb, s)
                      : launch_f8_v<FA, FB, 0>(A, B, C, M, N, K2, lda2, ldb2, ldc, sa, sb, s);
}
}  // namespace

// fp8 GEMM: C[M, N] (bf16) = sa[0] * sb[0] * A[M, K] . B[N, K]^T with A, B OCP fp8 (fa / fb: 0 = e4m3,
// 1 = e5m2).  K, lda, ldb in fp8 elements (bytes): K % 128 == 0, lda / ldb % 16 == 0; N % 8 == 0,
// ldc % 8 == 0; 16-B aligned base pointers.
ND_API int nd_gemm_nt_f8(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb,
                         int64_t ldc, int fa, int fb, const float* sa, const float* sb, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 128 || lda % 16 || ldb % 16 || N % 8 || ldc % 8 || lda < K || ldb < K ||
      (int64_t)TM * lda >= (1ll << 31) || (int64_t)TN * ldb >= (1ll << 31) || (int64_t)TM * ldc * 2 >= (1ll << 31) ||
      fa < 0 || fa > 1 || fb < 0 || fb > 1 || !sa || !sb)
    return (int)hipErrorInvalidValue;
  const int K2 = K / 2;
  const int64_t la = lda / 2, lb = ldb / 2;
  if (fa == 0 && fb == 0) return launch_f8<0, 0>(A, B, C, M, N, K2, la, lb, ldc, sa, sb, s);
  if (fa == 1 && fb == 0) return launch_f8<1, 0>(A, B, C, M, N, K2, la, lb, ldc, sa, sb, s);
  if (fa == 0 && fb == 1) return launch_f8<0, 1>(A, B, C, M, N, K2, la, lb, ldc, sa, sb, s);
  return launch_f8<1, 1>(A, B, C, M, N, K2, la, lb, ldc, sa, sb, s);
}

// GEMM schedule variant for A/B runs (see g_variant); returns the previous one
ND_API int nd_gemm_set_f8_variant(int v) {
  const int old = g_f8_variant;
  if (v >= -1 && v <= 3) g_f8_variant = v;
  return old;
}

ND_API int nd_gemm_set_group_m(int g) {
  const int old = g_group_m;
  if (g >= 0) g_group_m = g;
  return old;
}

