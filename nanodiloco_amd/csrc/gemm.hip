// Projection GEMM for gfx950 (forward and input-gradient GEMMs of every Llama projection, and the
// lm-head logits / dgrad):   C[M, N] = A[M, K] . B[N, K]^T   (both operands K-contiguous: tokens x in
// and a weight W[out, in] -- or its transposed copy W^T[in, out] for dgrad), bf16 in, fp32 accumulate.
//
// Geometry: 256 x 256 output tile per 512-thread workgroup, 8 waves as 2 (M) x 4 (N), 128 x 64 per
// wave = 8 x 4 v_mfma_f32_16x16x32_bf16 accumulators (128 AGPR/VGPR), BK = 64, one workgroup per CU
// (128 KiB LDS: two K-tile buffers of four 16-KiB half-tiles A0 | A1 | B0 | B1).
//
// Schedule (the "phase" pipeline): a K-tile is consumed in four phases; each phase =
//   [ds_read this phase's fragments] [LDS-DMA one half-tile of a LATER K-tile] s_barrier
//   lgkmcnt(0) setprio(1) 16 MFMAs (one 64 x 32 quadrant of the wave's 128 x 64, K = 64) setprio(0)
//   s_barrier
// Quadrant order and fragment reads: P1 reads B cols 0-31 + A rows 0-63 -> Q(lo, lo); P2 reads A rows
// 64-127 -> Q(hi, lo); P3 reads B cols 32-63 -> Q(hi, hi); P4 reads nothing -> Q(lo, hi).  So in tile t
// the A halves are last read in P2, the B halves in P3, and the DMA slots are
//   P1(t): B0(t+1)   P2(t): B1(t+1)   P3(t): A0(t+2)   P4(t): A1(t+2)
// (each half-tile is restaged at least one full phase -- two barriers -- after its last read: WAR-safe),
// and at the end of P4(t) one counted `s_waitcnt vmcnt(4)` retires all of tile t+1 while the two
// half-tiles of t+2 stay in flight across the barrier (RAW: a staged buffer is read only one phase
// after the wait + barrier that retire it).  The DMA never drains to 0 inside the loop.
//
// LDS-DMA (global_load_lds_dwordx4, 1 KiB = 8 rows x 128 B per wave-instruction) writes lane-linear
// LDS; the 16-B chunk index of row r is XOR-swizzled with (r >> 1) & 7 on the SOURCE address and on
// the ds_read_b128 fragment reads, which makes every ds_read_b128 lane group conflict-free.  The MFMA
// runs as B . A^T so each lane owns 4 consecutive output columns of one row (8-B bf16 stores), and
// pairs of columns 32 apart (RoPE halves at head_dim 64, gate/up of one SwiGLU unit) sit in one lane.
//
// Fused epilogues (each removes a separate HBM round trip of the [M, N] output):
//   EPI_STORE   C = bf16(acc)
//   EPI_ROPE    q|k|v projection: q and k heads rotated by RoPE (half-split, head_dim 32 / 64) on the
//               fp32 accumulator before the one bf16 rounding; v stored plainly (replaces rope_kernel)
//   EPI_SWIGLU  gate|up projection with interleaved weight rows (tile cols 0-31 of a wave = gate units
//               f..f+31, cols 32-63 = up units f..f+31): stores gu = [gate | up] (bf16, the backward's
//               input) AND act = silu(gate) * up (replaces swiglu_fwd)
//   EPI_DSWIGLU down-projection input gradient: acc = d(act); reads gate / up and stores
//               d(gate | up) (replaces swiglu_bwd and the d(act) tensor)
// XCD-aware workgroup order: consecutive output tiles (sharing an A row-panel) run on one XCD's L2.
#include "common.h"
#include <cstdlib>

using namespace nd;

namespace {
typedef __bf16 bfv8 __attribute__((ext_vector_type(8)));
constexpr int TM = 256, TN = 256, TK = 64;
constexpr int HALF = 128 * TK;  // elements of one half-tile (16 KiB)
constexpr int BUF = 4 * HALF;   // one K-tile: A0 A1 B0 B1 (64 KiB)

// s_waitcnt immediate (gfx9 encoding) for lgkmcnt(0) with vmcnt / expcnt left at their maxima
constexpr int LGKM0 = 0xC07F;

enum : int { EPI_STORE = 0, EPI_ROPE = 1, EPI_SWIGLU = 2, EPI_DSWIGLU = 3 };  // EPI_ROPE: HD = head_dim

struct Epi {
  // EPI_ROPE: fp32 tables [T, hd] (HF cat(freqs, freqs) layout; first half read), rotated columns
  const float* cosT;
  const float* sinT;
  int T, hd, rope_cols;
  // EPI_SWIGLU: act [M, F]; EPI_DSWIGLU: gu input [M, 2F] (ld_gu), output d(gate|up) is C (ldc)
  bf16_t* act;
  int64_t ld_act;
  const bf16_t* gu;
  int64_t ld_gu;
  int F;
};

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0, 0);
}

// one LDS-DMA wave-instruction: 64 lanes x 16 B from sbase + voff (per lane) to LDS [lds, lds + 1 KiB)
__device__ __forceinline__ void glds(const void* sbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}

// element offset of (row, k) in a [128][64] K-major half-tile (chunk swizzle (row >> 1) & 7)
__device__ __forceinline__ int koff(int row, int k) { return row * 64 + ((((k >> 3) ^ ((row >> 1) & 7))) << 3) + (k & 7); }

__device__ __forceinline__ bf16x8 frag(const bf16_t* half, int row, int kc) {
  return *reinterpret_cast<const bf16x8*>(&half[koff(row, kc)]);
}

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

template <int EPI, int HD, int SCHED>
__global__ void __launch_bounds__(512, 2) gemm_nt_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                         bf16_t* __restrict__ C, int M, int N, int K, int64_t lda,
                                                         int64_t ldb, int64_t ldc, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  // output-column tiles: 256 columns, except SWIGLU (128 gate/up units per tile, N = F)
  const int tcols = EPI == EPI_SWIGLU ? 128 : TN;
  const int tn = (N + tcols - 1) / tcols, tiles = ((M + TM - 1) / TM) * tn;
  const int id = xcd_remap(blockIdx.x, tiles);
  const int m0 = (id / tn) * TM, n0 = (id % tn) * tcols;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 2, wn = w & 3;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf16_t*)smem);

  // ---- per-thread DMA source offsets (bytes): half h, piece it -> tile row 128 h + 8 (w + 8 it) + lane / 8
  uint32_t va[2][2], vb[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int hr = 8 * (w + 8 * it) + (lane >> 3);  // row inside the half-tile
      const int lch = (lane & 7) ^ ((hr >> 1) & 7);   // logical 16-B chunk this lane fetches
      const int r = 128 * h + hr;                     // row inside the 256-row tile
      // offsets relative to the tile's first row (A + m0 lda, B + n0 ldb): 32-bit for any M, N
      int ar = m0 + r;
      ar = (ar < M ? ar : M - 1) - m0;  // tail rows: any valid row (their outputs are never stored)
      va[h][it] = (uint32_t)(((int64_t)ar * lda + lch * 8) * 2);
      int br;
      if (EPI == EPI_SWIGLU) {  // wave column group r / 64: 32 gate rows then the 32 matching up rows
        int f = n0 + (r >> 6) * 32 + (r & 31);
        f = f < N ? f : N - 1;
        br = ((r >> 5) & 1) * N + f;  // relative to B itself (gate and up rows are N apart)
      } else {
        br = n0 + r;
        br = (br < N ? br : N - 1) - n0;
      }
      vb[h][it] = (uint32_t)(((int64_t)br * ldb + lch * 8) * 2);
    }
  const int wr = __builtin_amdgcn_readfirstlane(w);
  const bf16_t* Ab = A + (int64_t)m0 * lda;
  const bf16_t* Bb = EPI == EPI_SWIGLU ? B : B + (int64_t)n0 * ldb;
  // stage half-tile `which` (0 A0, 1 A1, 2 B0, 3 B1) of K-tile kt into buffer kt & 1
  auto stage = [&](int kt, int which) {
    const uint32_t dst = lds0 + (uint32_t)(((kt & 1) * BUF + which * HALF) * 2);
    const bf16_t* base = (which < 2 ? Ab : Bb) + (int64_t)kt * TK;
    const int h = which & 1;
#pragma unroll
    for (int it = 0; it < 2; ++it)
      glds(base, which < 2 ? va[h][it] : vb[h][it], dst + (uint32_t)((wr + 8 * it) * 1024));
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / TK;
  if constexpr (SCHED == 0) {
  // prologue: tile 0 complete, A halves of tile 1 in flight
  stage(0, 0); stage(0, 1); stage(0, 2); stage(0, 3);
  if (nk > 1) {
    stage(1, 0); stage(1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  const int ar0 = lane & 15, kq = (lane >> 4) * 8;
  const int brow = (wn & 1) * 64 + (lane & 15);
  for (int kt = 0; kt < nk; ++kt) {
    const bf16_t* at = smem + (kt & 1) * BUF + wm * HALF;
    const bf16_t* bt = smem + (kt & 1) * BUF + (2 + (wn >> 1)) * HALF;
    bf16x8 fb[2][2], fa[4][2], fh[4][2];
    // ---------------- P1: B cols 0-31, A rows 0-63 -> quadrant (lo, lo); DMA B0(t+1)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fb[b][ks] = frag(bt, brow + b * 16, ks * 32 + kq);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fa[a][ks] = frag(at, a * 16 + ar0, ks * 32 + kq);
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) stage(kt + 1, 2);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) acc[a][b] = mfma16(fb[b][ks], fa[a][ks], acc[a][b]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---------------- P2: A rows 64-127 -> (hi, lo); DMA B1(t+1)
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fh[a][ks] = frag(at, 64 + a * 16 + ar0, ks * 32 + kq);
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) stage(kt + 1, 3);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) acc[4 + a][b] = mfma16(fb[b][ks], fh[a][ks], acc[4 + a][b]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---------------- P3: B cols 32-63 -> (hi, hi); DMA A0(t+2)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fb[b][ks] = frag(bt, brow + 32 + b * 16, ks * 32 + kq);
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 2 < nk) stage(kt + 2, 0);
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) acc[4 + a][2 + b] = mfma16(fb[b][ks], fh[a][ks], acc[4 + a][2 + b]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    // ---------------- P4: -> (lo, hi); DMA A1(t+2); retire tile t+1
    if (kt + 2 < nk) stage(kt + 2, 1);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) acc[a][2 + b] = mfma16(fb[b][ks], fa[a][ks], acc[a][2 + b]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  } else {
    // ---- SCHED 1: one barrier per K-tile, fragments double-buffered in registers: the reads of
    // k-step 1 (and of the next tile's k-step 0) are in flight under the MFMAs of the other k-step,
    // and the next tile's LDS-DMA has a whole K-tile of lead.
    stage(0, 0); stage(0, 1); stage(0, 2); stage(0, 3);
    if (nk > 1) {
      stage(1, 0); stage(1, 1); stage(1, 2); stage(1, 3);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int ar0 = lane & 15, kq = (lane >> 4) * 8;
    const int brow = (wn & 1) * 64 + (lane & 15);
    bf16x8 fa0[8], fb0[4], fa1[8], fb1[4];
    {
      const bf16_t* at = smem + wm * HALF;
      const bf16_t* bt = smem + (2 + (wn >> 1)) * HALF;
#pragma unroll
      for (int b = 0; b < 4; ++b) fb0[b] = frag(bt, brow + b * 16, kq);
#pragma unroll
      for (int a = 0; a < 8; ++a) fa0[a] = frag(at, a * 16 + ar0, kq);
    }
    for (int kt = 0; kt < nk; ++kt) {
      const bf16_t* at = smem + (kt & 1) * BUF + wm * HALF;
      const bf16_t* bt = smem + (kt & 1) * BUF + (2 + (wn >> 1)) * HALF;
      // k-step 0 fragments (read under the previous MFMAs) have landed.  The builtin form of the
      // wait is visible to the compiler's counter tracking: without it, 24 outstanding LDS reads
      // exceed the 4-bit lgkmcnt and it would drain to 0 right before the MFMAs below.
      __builtin_amdgcn_s_waitcnt(LGKM0);
#pragma unroll
      for (int b = 0; b < 4; ++b) fb1[b] = frag(bt, brow + b * 16, 32 + kq);
#pragma unroll
      for (int a = 0; a < 8; ++a) fa1[a] = frag(at, a * 16 + ar0, 32 + kq);
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = mfma16(fb0[b], fa0[a], acc[a][b]);
      __builtin_amdgcn_sched_barrier(0);
      // retire tile kt+1 (the only DMA in flight) and this wave's reads of buffer kt & 1
      if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_waitcnt(LGKM0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 2 < nk) { stage(kt + 2, 0); stage(kt + 2, 1); stage(kt + 2, 2); stage(kt + 2, 3); }
      if (kt + 1 < nk) {
        const bf16_t* an = smem + ((kt + 1) & 1) * BUF + wm * HALF;
        const bf16_t* bn = smem + ((kt + 1) & 1) * BUF + (2 + (wn >> 1)) * HALF;
#pragma unroll
        for (int b = 0; b < 4; ++b) fb0[b] = frag(bn, brow + b * 16, kq);
#pragma unroll
        for (int a = 0; a < 8; ++a) fa0[a] = frag(an, a * 16 + ar0, kq);
      }
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = mfma16(fb1[b], fa1[a], acc[a][b]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // ---------------- epilogue: acc[a][b] lane l reg r = C[m0 + wm*128 + a*16 + (l & 15)][col(b) + 4 (l >> 4) + r]
  const int q4 = 4 * (lane >> 4);
  if (EPI == EPI_STORE || EPI == EPI_ROPE) {
    const int nb = n0 + wn * 64;  // this wave's 64 output columns
    // RoPE (compile-time head_dim HD): column c = 16 b + 4q + r of the wave's group pairs with c + HD/2
    // of the same head -- n-tile b + HD/32, the same lane (all indices static: no scratch)
    constexpr int HALFD = HD / 2;
    bool rot[4] = {false, false, false, false};
    if constexpr (EPI == EPI_ROPE) {
#pragma unroll
      for (int b = 0; b < 4; ++b) rot[b] = ((b * 16) % HD) < HALFD && (nb + b * 16) < ep.rope_cols;
    }
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      const int m = m0 + wm * 128 + a * 16 + (lane & 15);
      if (m >= M) continue;
      f32x4 v[4] = {acc[a][0], acc[a][1], acc[a][2], acc[a][3]};
      if constexpr (EPI == EPI_ROPE) {
        const int t = m % ep.T;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          if (((b * 16) % HD) >= HALFD) continue;  // static: b is the first half of its head
          const int p = (b + HALFD / 16) & 3;
          if (!rot[b]) continue;
          const int i = (b * 16) % HD + q4;
          const float4 c = *reinterpret_cast<const float4*>(ep.cosT + (int64_t)t * HD + i);
          const float4 s = *reinterpret_cast<const float4*>(ep.sinT + (int64_t)t * HD + i);
          const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x1 = acc[a][b][r], x2 = acc[a][p][r];
            v[b][r] = x1 * cc[r] - x2 * ss[r];
            v[p][r] = x2 * cc[r] + x1 * ss[r];
          }
        }
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int n = nb + b * 16 + q4;
        if (n >= N) continue;
        uint2 o;
        o.x = pack2(v[b][0], v[b][1]);
        o.y = pack2(v[b][2], v[b][3]);
        *reinterpret_cast<uint2*>(C + (int64_t)m * ldc + n) = o;
      }
    }
  } else if (EPI == EPI_SWIGLU) {
    // lane's gate units f = n0 + wn*32 + 16 b + 4q + r (b = 0, 1) pair with up = acc[a][b + 2]
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      const int m = m0 + wm * 128 + a * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int f = n0 + wn * 32 + b * 16 + q4;
        if (f >= N) continue;
        uint2 g, u, y;
        g.x = pack2(acc[a][b][0], acc[a][b][1]);
        g.y = pack2(acc[a][b][2], acc[a][b][3]);
        u.x = pack2(acc[a][b + 2][0], acc[a][b + 2][1]);
        u.y = pack2(acc[a][b + 2][2], acc[a][b + 2][3]);
        // act from the rounded gate / up: exactly what the backward will see
        y.x = pack2(silu(lo_bf(g.x)) * lo_bf(u.x), silu(hi_bf(g.x)) * hi_bf(u.x));
        y.y = pack2(silu(lo_bf(g.y)) * lo_bf(u.y), silu(hi_bf(g.y)) * hi_bf(u.y));
        bf16_t* crow = C + (int64_t)m * ldc;
        *reinterpret_cast<uint2*>(crow + f) = g;
        *reinterpret_cast<uint2*>(crow + N + f) = u;
        *reinterpret_cast<uint2*>(ep.act + (int64_t)m * ep.ld_act + f) = y;
      }
    }
  } else {  // EPI_DSWIGLU: acc = d(act)[m][f]; C = d(gate | up) [M, 2N]
    const int nb = n0 + wn * 64;
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      const int m = m0 + wm * 128 + a * 16 + (lane & 15);
      if (m >= M) continue;
      const bf16_t* grow = ep.gu + (int64_t)m * ep.ld_gu;
      bf16_t* crow = C + (int64_t)m * ldc;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int f = nb + b * 16 + q4;
        if (f >= N) continue;
        const uint2 g2 = *reinterpret_cast<const uint2*>(grow + f);
        const uint2 u2 = *reinterpret_cast<const uint2*>(grow + N + f);
        const float g[4] = {lo_bf(g2.x), hi_bf(g2.x), lo_bf(g2.y), hi_bf(g2.y)};
        const float u[4] = {lo_bf(u2.x), hi_bf(u2.x), lo_bf(u2.y), hi_bf(u2.y)};
        float dg[4], du[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = acc[a][b][r];
          const float sg = 1.f / (1.f + __expf(-g[r]));
          du[r] = d * g[r] * sg;
          dg[r] = d * u[r] * sg * (1.f + g[r] * (1.f - sg));
        }
        *reinterpret_cast<uint2*>(crow + f) = make_uint2(pack2(dg[0], dg[1]), pack2(dg[2], dg[3]));
        *reinterpret_cast<uint2*>(crow + N + f) = make_uint2(pack2(du[0], du[1]), pack2(du[2], du[3]));
      }
    }
  }
}

// SCHED 0: four barrier-separated phases per K-tile; SCHED 1 (default): register-pipelined, one
// barrier per K-tile.  ND_GEMM_SCHED selects one for A/B runs.
inline int sched_choice() {
  static const int v = [] {
    const char* e = getenv("ND_GEMM_SCHED");
    return e ? atoi(e) : 1;
  }();
  return v;
}

template <int EPI, int HD, int SCHED>
int launch_s(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
             const Epi& ep, hipStream_t s) {
  const size_t lds = 2 * (size_t)BUF * sizeof(bf16_t);  // 128 KiB
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<EPI, HD, SCHED>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return (int)attr;
  const int tcols = EPI == EPI_SWIGLU ? 128 : TN;
  const int tiles = ((M + TM - 1) / TM) * ((N + tcols - 1) / tcols);
  hipLaunchKernelGGL((gemm_nt_kernel<EPI, HD, SCHED>), dim3(tiles), dim3(512), lds, s, (const bf16_t*)A,
                     (const bf16_t*)B, (bf16_t*)C, M, N, K, lda, ldb, ldc, ep);
  ND_LAUNCH_CHECK();
}

template <int EPI, int HD = 64>
int launch(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
           const Epi& ep, hipStream_t s) {
  return sched_choice() == 0 ? launch_s<EPI, HD, 0>(A, B, C, M, N, K, lda, ldb, ldc, ep, s)
                             : launch_s<EPI, HD, 1>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
}

bool shapes_ok(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc) {
  // byte offsets of one operand tile stay 32-bit (per-lane DMA offsets)
  return M > 0 && N > 0 && K > 0 && K % TK == 0 && N % 4 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0 &&
         lda >= K && ldb >= K && (int64_t)TM * lda * 2 < (1ll << 31) && (int64_t)TN * ldb * 2 < (1ll << 31);
}
}  // namespace

// C[M, N] = A[M, K] . B[N, K]^T (bf16 in / out, fp32 accumulate).  K % 64 == 0, N % 4 == 0,
// lda / ldb % 8 == 0, ldc % 4 == 0, 16-B aligned base pointers.
ND_API int nd_gemm_nt(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb,
                      int64_t ldc, hipStream_t s) {
  if (!shapes_ok(M, N, K, lda, ldb, ldc)) return (int)hipErrorInvalidValue;
  Epi ep{};
  return launch<EPI_STORE>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
}

// q|k|v projection with RoPE on the first rope_cols columns (q and k heads): rows are tokens
// (t = row % T), tables fp32 [T, hd].  hd in {32, 64}.
ND_API int nd_gemm_nt_rope(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb,
                           int64_t ldc, const float* cosT, const float* sinT, int T, int hd, int rope_cols,
                           hipStream_t s) {
  if (!shapes_ok(M, N, K, lda, ldb, ldc) || (hd != 32 && hd != 64) || rope_cols % hd || T <= 0)
    return (int)hipErrorInvalidValue;
  Epi ep{};
  ep.cosT = cosT; ep.sinT = sinT; ep.T = T; ep.hd = hd; ep.rope_cols = rope_cols;
  return hd == 64 ? launch<EPI_ROPE, 64>(A, B, C, M, N, K, lda, ldb, ldc, ep, s)
                  : launch<EPI_ROPE, 32>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
}

// gate|up projection + SwiGLU: B = fused weight [2F, K] (gate rows then up rows), gu = C [M, 2F]
// (ldc), act [M, F] (ld_act).  F % 4 == 0.
ND_API int nd_gemm_nt_swiglu(const void* A, const void* B, void* gu, void* act, int M, int F, int K, int64_t lda,
                             int64_t ldb, int64_t ldc, int64_t ld_act, hipStream_t s) {
  if (!shapes_ok(M, F, K, lda, ldb, ldc) || ldc < 2 * (int64_t)F || ld_act % 4 ||
      (int64_t)2 * F * ldb * 2 >= (1ll << 31))  // per-lane DMA offsets span both weight halves
    return (int)hipErrorInvalidValue;
  Epi ep{};
  ep.act = (bf16_t*)act; ep.ld_act = ld_act; ep.F = F;
  return launch<EPI_SWIGLU>(A, B, gu, M, F, K, lda, ldb, ldc, ep, s);
}

// down-projection input gradient fused with the SwiGLU backward: d(act) = A . B^T (A = dY [M, K],
// B = W_down^T [F, K]) is never stored; reads gu [M, 2F] and writes dgu [M, 2F].
ND_API int nd_gemm_nt_dswiglu(const void* A, const void* B, const void* gu, void* dgu, int M, int F, int K,
                              int64_t lda, int64_t ldb, int64_t ld_gu, int64_t ld_dgu, hipStream_t s) {
  if (!shapes_ok(M, F, K, lda, ldb, ld_dgu) || ld_gu % 4 || ld_gu < 2 * (int64_t)F || ld_dgu < 2 * (int64_t)F)
    return (int)hipErrorInvalidValue;
  Epi ep{};
  ep.gu = (const bf16_t*)gu; ep.ld_gu = ld_gu; ep.F = F;
  return launch<EPI_DSWIGLU>(A, B, dgu, M, F, K, lda, ldb, ld_dgu, ep, s);
}
