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
#include <type_traits>

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

// the same piece through a buffer descriptor (buffer_load_dwordx4 ... offen lds): 32-bit per-lane
// offsets against a wave-uniform base in four SGPRs
__device__ __forceinline__ void glds_buf(__amdgpu_buffer_rsrc_t rsrc, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_n(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// bf16-pack the 4-column quads of two adjacent 16-column blocks (x = block b, y = block b + 1) and
// v_permlane16_swap them so lane rows 0 / 2 hold 8 consecutive columns of block b and rows 1 / 3
// those of block b + 1 (rows 0 / 1: columns 0-7, rows 2 / 3: columns 8-15)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 pair16(const f32x4& x, const f32x4& y) {
  const auto s0 = __builtin_amdgcn_permlane16_swap(pack2(x[0], x[1]), pack2(y[0], y[1]), false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(pack2(x[2], x[3]), pack2(y[2], y[3]), false, false);
  u32x4 d = u32x4{s0[0], s1[0], s0[1], s1[1]};
  asm volatile("s_nop 1" : "+v"(d));  // permlane result -> store data: keep two wait states
  return d;
}
__device__ __forceinline__ float round_bf(float x) { return lo_bf(pack2(x, 0.f)); }
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7FFFFFFF, 0x00020000);
}

// element offset of (row, k) in a [128][64] K-major half-tile (chunk swizzle (row >> 1) & 7)
__device__ __forceinline__ int koff(int row, int k) { return row * 64 + ((((k >> 3) ^ ((row >> 1) & 7))) << 3) + (k & 7); }

__device__ __forceinline__ bf16x8 frag(const bf16_t* half, int row, int kc) {
  return *reinterpret_cast<const bf16x8*>(&half[koff(row, kc)]);
}

// chunk swizzle of the 4-wave kernel: SWZ 0 = (row >> 1) & 7 (conflict-free ds_read_b128, but the
// LDS-DMA source order inside a 64-B half is permuted); SWZ 1 = swap the two 64-B halves of odd
// row pairs only (each lane quad reads 64 ascending contiguous bytes; 2-way read conflicts)
template <int SWZ>
__device__ __forceinline__ int swz(int row) { return SWZ == 0 ? ((row >> 1) & 7) : (((row >> 1) & 1) << 2); }
// SWZ 2: padded block layout.  A half-tile is 16 LDS blocks of 1056 B (8 rows x 128 B + 32 B pad);
// block b holds rows b, b + 16, ..., b + 112 unswizzled, so every LDS-DMA lane octet reads one whole
// 128-B row in ascending order (one cache access per line), and a ds_read_b128 lane group (16 rows
// 16 apart in block index) lands on 16 distinct 16-B bank slots thanks to the 32-B pad.
constexpr int BLOCK_P = 1056;                 // bytes per padded block
constexpr int HALF_P = 16 * BLOCK_P / 2;      // elements per padded half-tile
template <int SWZ>
__device__ __forceinline__ bf16x8 fragz(const bf16_t* half, int row, int kc) {
  if constexpr (SWZ == 2)
    return *reinterpret_cast<const bf16x8*>(&half[(row & 15) * (BLOCK_P / 2) + (row >> 4) * 64 + kc]);
  return *reinterpret_cast<const bf16x8*>(&half[row * 64 + (((kc >> 3) ^ swz<SWZ>(row)) << 3) + (kc & 7)]);
}

// the same MFMA with the accumulator pinned to AGPRs (tied "+a" operand): hipcc's register allocator
// otherwise rotates a 256-register accumulator set through VGPR copies every K-step.  The chain on
// one accumulator needs no wait states; readers of the result wait for `mfma_drain()`.
__device__ __forceinline__ void mfma16a(const bf16x8& a, const bf16x8& b, f32x4& c) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_drain() { asm volatile("s_nop 15\n\ts_nop 3" ::: "memory"); }

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


// =====================================================================================================
// Variant 2 / 3: four waves (256 threads), each wave a 128 x 128 quadrant of the 256 x 256 tile
// (8 x 8 v_mfma_f32_16x16x32_bf16 accumulators = 256 AGPRs), one wave per SIMD: no partner wave
// competing for the SIMD's matrix pipe, and 32 ds_read_b128 per 128 MFMAs (vs 24 per 64 with the
// 8-wave 128 x 64 split).  Same LDS image (two 64-KiB K-tile buffers of four swizzled half-tiles),
// fragments double-buffered in registers, one barrier per K-tile.
// PERSIST (variant 3): one workgroup per CU walks tiles first, first + G, ... (XCD-remapped so the
// 32 workgroups of one XCD work on neighbouring tiles); the LDS-DMA stream runs ACROSS tile
// boundaries, so the next tile's first K-tiles land while this tile's epilogue stores drain.
template <int EPI, int HD, bool PERSIST, int SWZ, int ABL = 0, int LD = 0, int STP = 0>
__global__ void __launch_bounds__(256, 1) gemm4_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                       bf16_t* __restrict__ C, int M, int N, int K, int64_t lda,
                                                       int64_t ldb, int64_t ldc, Epi ep, int GM) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  constexpr int tcols = EPI == EPI_SWIGLU ? 128 : TN;
  constexpr int HS = SWZ == 2 ? HALF_P : HALF;  // elements per half-tile
  constexpr int BS = 4 * HS;                     // elements per K-tile buffer
  const int tn = (N + tcols - 1) / tcols, tiles = ((M + TM - 1) / TM) * tn;
  const int G = gridDim.x;
  const int first = PERSIST ? xcd_remap(blockIdx.x, G) : xcd_remap(blockIdx.x, tiles);
  const int my_tiles = PERSIST ? (first < tiles ? (tiles - 1 - first) / G + 1 : 0) : 1;
  const int nk = K / TK;
  const int total = my_tiles * nk;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int wr = __builtin_amdgcn_readfirstlane(w);
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf16_t*)smem);

  // ---- staging stream state (runs up to two K-tiles ahead of the compute stream)
  int s_tile = first, s_kt = 0;
  const int tmn = (M + TM - 1) / TM;
  // tile t -> (m, n): groups of GM m-panels walked n-major inside the group, so the 32 concurrent
  // tiles of one XCD form a compact GM x (32 / GM) block (fewer distinct A / B K-slices per step)
  auto coords = [&](int t, int& m0, int& n0) __attribute__((always_inline)) {
    if (GM <= 1) {
      m0 = (t / tn) * TM;
      n0 = (t % tn) * tcols;
    } else {
      const int per = GM * tn, grp = t / per, r = t - grp * per;
      const int gm = (tmn - grp * GM) < GM ? (tmn - grp * GM) : GM;  // last group may be short
      m0 = (grp * GM + r % gm) * TM;
      n0 = (r / gm) * tcols;
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
        // SWZ 2: piece p of wave w is LDS block b = w + 4p holding rows b, b + 16, ..., b + 112
        const int hr = SWZ == 2 ? (w + 4 * p) + 16 * (lane >> 3) : 8 * (w + 4 * p) + (lane >> 3);
        const int lch = SWZ == 2 ? (lane & 7) : (lane & 7) ^ swz<SWZ>(hr);
        const int r = 128 * h + hr;
        int ar = s_m0 + r;
        ar = (ar < M ? ar : M - 1) - s_m0;
        va[h][p] = (uint32_t)(((int64_t)ar * lda + lch * 8) * 2);
        int br;
        if (EPI == EPI_SWIGLU) {  // wave column group r / 128: 64 gate rows then the 64 matching up rows
          int f = s_n0 + (r >> 7) * 64 + (r & 63);
          f = f < N ? f : N - 1;
          br = ((r >> 6) & 1) * N + f;
        } else {
          br = s_n0 + r;
          br = (br < N ? br : N - 1) - s_n0;
        }
        vb[h][p] = (uint32_t)(((int64_t)br * ldb + lch * 8) * 2);
      }
  };
  offsets();
  // stage the next K-tile of the staging stream into buffer `buf`, advance the stream
  // LDS-DMA piece j (0-7: A half j / 4, 8-15: B half (j - 8) / 4) of the staging stream's current
  // K-tile into buffer `buf`; advance() moves the stream to its next K-tile
  auto stage_piece = [&](int buf, int j) __attribute__((always_inline)) {
    const uint32_t dst = lds0 + (uint32_t)(buf * BS * 2);
    const int h = (j >> 2) & 1, p = j & 3;
    constexpr int PIECE = SWZ == 2 ? BLOCK_P : 1024;  // bytes between a wave's consecutive pieces
    if (j < 8) {
      const bf16_t* Ab = A + (int64_t)s_m0 * lda + (int64_t)s_kt * TK;
      const uint32_t d = dst + (uint32_t)((h * HS) * 2 + (wr + 4 * p) * PIECE);
      if constexpr (LD == 1) glds_buf(make_rsrc(Ab), va[h][p], d);
      else glds(Ab, va[h][p], d);
    } else {
      const bf16_t* Bb = (EPI == EPI_SWIGLU ? B : B + (int64_t)s_n0 * ldb) + (int64_t)s_kt * TK;
      const uint32_t d = dst + (uint32_t)(((2 + h) * HS) * 2 + (wr + 4 * p) * PIECE);
      if constexpr (LD == 1) glds_buf(make_rsrc(Bb), vb[h][p], d);
      else glds(Bb, vb[h][p], d);
    }
  };
  auto advance = [&]() __attribute__((always_inline)) {
    if (++s_kt == nk) {
      s_kt = 0;
      s_tile += G;
      if (PERSIST && s_tile < tiles) {
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

  f32x4 acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (total == 0) return;

  stage_next(0);
  if (total > 1) {
    stage_next(1);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  const int ar0 = lane & 15, kq = (lane >> 4) * 8;
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  {
    const bf16_t* at = smem + wm * HS;
    const bf16_t* bt = smem + (2 + wn) * HS;
#pragma unroll
    for (int b = 0; b < 8; ++b) fb0[b] = fragz<SWZ>(bt, b * 16 + ar0, kq);
#pragma unroll
    for (int a = 0; a < 8; ++a) fa0[a] = fragz<SWZ>(at, a * 16 + ar0, kq);
  }
  for (int lt = 0; lt < my_tiles; ++lt) {
  for (int kt = 0; kt < nk; ++kt) {
    const int g = lt * nk + kt;  // position in the workgroup's K-tile stream
    const int buf = g & 1;
    const bool more1 = g + 1 < total, more2 = g + 2 < total;
    const bf16_t* at = smem + buf * BS + wm * HS;
    const bf16_t* bt = smem + buf * BS + (2 + wn) * HS;
    __builtin_amdgcn_s_waitcnt(LGKM0);
    // k-step 0: per row block a, 8 MFMAs with this step's fragments; the two k-step-1 fragment
    // reads of block a ride under them
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      if (!(ABL & 2)) {
        fb1[a] = fragz<SWZ>(bt, a * 16 + ar0, 32 + kq);
        fa1[a] = fragz<SWZ>(at, a * 16 + ar0, 32 + kq);
      } else if (a == 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i) { fb1[i] = fb0[i]; fa1[i] = fa0[i]; }
      }
#pragma unroll
      for (int b = 0; b < 8; ++b) mfma16a(fb0[b], fa0[a], acc[a][b]);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (more1 && !(ABL & 1)) {
      // K-tile g + 1 must have landed.  Right after an epilogue its (fixed number of) stores were
      // issued after that DMA and may stay in flight
      if (EPI != EPI_DSWIGLU && kt == 0 && lt > 0) {
        // (K-tile g + 1 was staged during the previous tile's last k-step, before those stores)
        if constexpr (EPI == EPI_SWIGLU) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __builtin_amdgcn_s_waitcnt(LGKM0);
    if (!(ABL & 4)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    // k-step 1: two LDS-DMA pieces of K-tile g + 2 (into the buffer just released) and two
    // fragment reads of K-tile g + 1 per 8 MFMAs: an LDS-DMA issue stalls the wave for ~100
    // cycles, hidden behind the MFMAs already in the pipe (a burst of 16 would idle the SIMD)
    const bf16_t* an = smem + (buf ^ 1) * BS + wm * HS;
    const bf16_t* bn = smem + (buf ^ 1) * BS + (2 + wn) * HS;
    // (the C epilogue stages through its own LDS region, so the stream never pauses at a tile end)
    const bool stage_now = more2;
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      if (stage_now && !(ABL & 1) && LD != 2) {  // ABL: ablation builds for profiling only (wrong results)
        stage_piece(buf, a);
        stage_piece(buf, 8 + a);
      }
      if (!(ABL & 2)) {
        fb0[a] = fragz<SWZ>(bn, a * 16 + ar0, kq);  // past the stream's end: reads unused LDS
        fa0[a] = fragz<SWZ>(an, a * 16 + ar0, kq);
      }
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        mfma16a(fb1[b], fa1[a], acc[a][b]);
        // LD 2: the group's two DMA pieces after its 2nd and 6th MFMA (issue stalls overlap MFMAs)
        if (LD == 2 && stage_now && (b == 1 || b == 5)) stage_piece(buf, (b == 1 ? 0 : 8) + a);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (stage_now) advance();
  }
    mfma_drain();
    const int c_tile = first + lt * G;
    // ---------------- epilogue of tile c_tile
    int m0, n0;
    coords(c_tile, m0, n0);
    const int q4 = 4 * (lane >> 4);
    if constexpr ((ABL & 8) != 0) {  // ablation: no epilogue stores (keep the accumulators live)
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) asm volatile("" ::"a"(acc[a][b]));
    } else if (EPI == EPI_STORE || EPI == EPI_ROPE) {
      // C through the wave's own LDS staging region (behind the two K-tile buffers, so the DMA
      // stream runs on), 16 rows of the wave's 128 x 128 quadrant per pass: v_permlane16_swap pairs the 4-column quads of blocks
      // b, b + 1 into 16-B pieces (ds_write_b128, rows padded to 272 B), then 16 lanes per row read
      // back whole 256-B row segments and store them with buffer_store_dwordx4 -- full 128-B lines
      // per store instead of 16 half-lines.  Out-of-range lanes are dropped by the descriptor (rows
      // past M) or an offset sentinel (columns past N), so every wave issues exactly 32 stores.
      const __amdgpu_buffer_rsrc_t crs = make_rsrc_n(C + (int64_t)m0 * ldc, (uint32_t)((int64_t)(M - m0 < TM ? M - m0 : TM) * ldc * 2));
      const int q = lane >> 4;
      constexpr int RS = 136;  // staging row stride (elements): 256 B + 16 B pad
      bf16_t* cst = smem + 2 * BS + w * (16 * RS);
      const int ccol = n0 + wn * 128 + (lane & 15) * 8;  // read-back: this lane's 8 columns
      const uint32_t coff = ccol < N ? (uint32_t)(ccol * 2) : 0x80000000u;
      constexpr int HALFD = HD / 2;
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        {
          // per group of 4 column blocks (one 64-wide head, or two 32-wide ones): RoPE pairs
          // block b with b + HD/32 inside the group; the tables repeat every head
          float4 ct[2], st[2];
          if constexpr (EPI == EPI_ROPE) {
            const int t = (m0 + wm * 128 + a * 16 + (lane & 15)) % ep.T;
#pragma unroll
            for (int j = 0; j < HALFD / 16; ++j) {
              ct[j] = *reinterpret_cast<const float4*>(ep.cosT + (int64_t)t * HD + j * 16 + q4);
              st[j] = *reinterpret_cast<const float4*>(ep.sinT + (int64_t)t * HD + j * 16 + q4);
            }
          }
#pragma unroll
          for (int g4 = 0; g4 < 2; ++g4) {
            f32x4 v[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) v[b] = acc[a][g4 * 4 + b];
            if constexpr (EPI == EPI_ROPE) {
              // q / k columns rotate (rope_cols % HD == 0); v columns pass through (branch-free:
              // a wave-uniform branch here made hipcc spill the accumulator set)
              const bool rot = n0 + wn * 128 + g4 * 64 < ep.rope_cols;
#pragma unroll
              for (int b = 0; b < 4; ++b) {
                if (((b * 16) % HD) >= HALFD) continue;  // static: b is in the first half of its head
                const int p = b + HALFD / 16, j = ((b * 16) % HD) / 16;
                const float cc[4] = {ct[j].x, ct[j].y, ct[j].z, ct[j].w};
                const float ss[4] = {st[j].x, st[j].y, st[j].z, st[j].w};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const float c1 = rot ? cc[r] : 1.f, s1 = rot ? ss[r] : 0.f;
                  const float x1 = v[b][r], x2 = v[p][r];
                  v[b][r] = x1 * c1 - x2 * s1;
                  v[p][r] = x2 * c1 + x1 * s1;
                }
              }
            }
#pragma unroll
            for (int b = 0; b < 4; b += 2) {
              const int col = (g4 * 4 + b + (q & 1)) * 16 + (q >> 1) * 8;
              *reinterpret_cast<u32x4*>(cst + (lane & 15) * RS + col) = pair16(v[b], v[b + 1]);
            }
          }
        }
        asm volatile("" ::: "memory");  // cross-lane LDS exchange: no compiler reordering
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = i * 4 + q;  // 0..15 inside this pass
          const u32x4 d = *reinterpret_cast<const u32x4*>(cst + row * RS + (lane & 15) * 8);
          const int mr = wm * 128 + a * 16 + row;
          __builtin_amdgcn_raw_buffer_store_b128(d, crs, coff == 0x80000000u ? coff : coff + (uint32_t)(mr * ldc * 2), 0, STP);
        }
        asm volatile("" ::: "memory");
      }
    } else if (EPI == EPI_SWIGLU) {
      const __amdgpu_buffer_rsrc_t crs = make_rsrc_n(C + (int64_t)m0 * ldc, (uint32_t)((int64_t)(M - m0 < TM ? M - m0 : TM) * ldc * 2));
      const __amdgpu_buffer_rsrc_t ars = make_rsrc_n(ep.act + (int64_t)m0 * ep.ld_act, (uint32_t)((int64_t)(M - m0 < TM ? M - m0 : TM) * ep.ld_act * 2));
      const int q = lane >> 4;
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const int mr = wm * 128 + a * 16 + (lane & 15);
#pragma unroll
        for (int b = 0; b < 4; b += 2) {
          // gate / up rounded to bf16 first: act is computed from exactly what the backward reads
          f32x4 g2[2], u2[2], y2[2];
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              g2[j][r] = round_bf(acc[a][b + j][r]);
              u2[j][r] = round_bf(acc[a][b + j + 4][r]);
              y2[j][r] = silu(g2[j][r]) * u2[j][r];
            }
          const int f = n0 + wn * 64 + (b + (q & 1)) * 16 + (q >> 1) * 8;
          const bool ok = f < N;
          const uint32_t og = ok ? (uint32_t)(((int64_t)mr * ldc + f) * 2) : 0x80000000u;
          const uint32_t ou = ok ? (uint32_t)(((int64_t)mr * ldc + N + f) * 2) : 0x80000000u;
          const uint32_t oy = ok ? (uint32_t)(((int64_t)mr * ep.ld_act + f) * 2) : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b128(pair16(g2[0], g2[1]), crs, og, 0, STP);
          __builtin_amdgcn_raw_buffer_store_b128(pair16(u2[0], u2[1]), crs, ou, 0, STP);
          __builtin_amdgcn_raw_buffer_store_b128(pair16(y2[0], y2[1]), ars, oy, 0, STP);
        }
      }
    } else {  // EPI_DSWIGLU
      const int nb = n0 + wn * 128;
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const int m = m0 + wm * 128 + a * 16 + (lane & 15);
        if (m >= M) continue;
        const bf16_t* grow = ep.gu + (int64_t)m * ep.ld_gu;
        bf16_t* crow = C + (int64_t)m * ldc;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const int f = nb + b * 16 + q4;
          if (f >= N) continue;
          const uint2 g2 = *reinterpret_cast<const uint2*>(grow + f);
          const uint2 u2 = *reinterpret_cast<const uint2*>(grow + N + f);
          const float gv[4] = {lo_bf(g2.x), hi_bf(g2.x), lo_bf(g2.y), hi_bf(g2.y)};
          const float uv[4] = {lo_bf(u2.x), hi_bf(u2.x), lo_bf(u2.y), hi_bf(u2.y)};
          float dg[4], du[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = acc[a][b][r];
            const float sg = 1.f / (1.f + __expf(-gv[r]));
            du[r] = d * gv[r] * sg;
            dg[r] = d * uv[r] * sg * (1.f + gv[r] * (1.f - sg));
          }
          *reinterpret_cast<uint2*>(crow + f) = make_uint2(pack2(dg[0], dg[1]), pack2(dg[2], dg[3]));
          *reinterpret_cast<uint2*>(crow + N + f) = make_uint2(pack2(du[0], du[1]), pack2(du[2], du[3]));
        }
      }
    }
    if (PERSIST) {
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

// ---------------------------------------------------------------------------------------------
// fp8 x fp8 -> bf16 projection GEMM (the --fp8 recipe's forward e4m3 x e4m3 and input-gradient
// e5m2 x e4m3 GEMMs; replaces torch._scaled_mm).  C = bf16(sa * sb * A . B^T), sa / sb device scalars
// (the recipe's inverse scales: delayed scaling, no host sync).
//
// A K-tile of 128 fp8 = 128 B per row is byte-for-byte the bf16 kernel's 64-element K-tile, so the
// LDS image, the LDS-DMA staging stream (persistent grid, padded block layout) and the C epilogue
// path are those of gemm4_kernel<.., PERSIST, SWZ 2>; the operands are addressed as bf16 pairs.
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
int g_variant = [] {
  const char* e = getenv("ND_GEMM_VARIANT");
  return e ? atoi(e) : 10;
}();

// tile grouping of the 4-wave kernels (see coords()); ND_GEMM_GROUP_M or nd_gemm_set_group_m
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

template <int EPI, int HD, int SCHED>
int launch_s(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
             const Epi& ep, hipStream_t s) {
  // two K-tile buffers (128 / 132 KiB) + the C epilogue's staging rows (4 waves x 16 x 272 B)
  const size_t lds = (2 * (size_t)(SCHED >= 5 ? 4 * HALF_P : BUF) + 4 * 16 * 136) * sizeof(bf16_t);
  const int tcols = EPI == EPI_SWIGLU ? 128 : TN;
  const int tiles = ((M + TM - 1) / TM) * ((N + tcols - 1) / tcols);
  if constexpr (SCHED <= 1) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<EPI, HD, SCHED>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (attr != hipSuccess) return (int)attr;
    hipLaunchKernelGGL((gemm_nt_kernel<EPI, HD, SCHED>), dim3(tiles), dim3(512), lds, s, (const bf16_t*)A,
                       (const bf16_t*)B, (bf16_t*)C, M, N, K, lda, ldb, ldc, ep);
  } else {
    constexpr bool P = SCHED >= 3 && SCHED != 7 && SCHED != 8 && SCHED != 9;  // 10: persistent, padded, interleaved DMA
    constexpr int Z = SCHED == 4 ? 1 : SCHED >= 5 ? 2 : 0;
    constexpr int STPC = SCHED == 9 ? 0 : 2;  // C-store cache policy: nt (aux 2; +5 % over plain stores, profiles/r2_gemm_ab.md); 9 = plain (A/B)
    constexpr int AB = SCHED > 10 ? SCHED - 10 : 0;  // ablation builds (profiling only)
    constexpr int LDK = SCHED == 6 ? 1 : SCHED == 10 ? 2 : 0;  // 1: buffer_load ... lds; 2: DMA pieces between MFMAs
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm4_kernel<EPI, HD, P, Z, AB, LDK, STPC>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (attr != hipSuccess) return (int)attr;
    const int grid = P ? (tiles < num_cus() ? tiles : num_cus()) : tiles;
    hipLaunchKernelGGL((gemm4_kernel<EPI, HD, P, Z, AB, LDK, STPC>), dim3(grid), dim3(256), lds, s, (const bf16_t*)A,
                       (const bf16_t*)B, (bf16_t*)C, M, N, K, lda, ldb, ldc, ep, g_group_m);
  }
  ND_LAUNCH_CHECK();
}

template <int EPI, int HD = 64>
int launch(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
           const Epi& ep, hipStream_t s) {
  // the 4-wave kernels store 8-column (16-B) pieces and keep per-tile byte offsets 32-bit
  // EPI_ROPE stays on the 8-wave kernel: its epilogue's register pressure makes hipcc move the
  // accumulators between AGPRs, and an inline-asm MFMA's result must not be touched by compiler
  // code before it lands (wrong values measured; tests/test_gemm_gpu.py rope cases)
  const bool four_ok = EPI != EPI_ROPE && N % 8 == 0 && ldc % 8 == 0 && (int64_t)TM * ldc * 2 < (1ll << 31) &&
                       (EPI != EPI_SWIGLU || ep.ld_act % 8 == 0);
  if constexpr (EPI == EPI_ROPE) return launch_s<EPI, HD, 1>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
  switch (four_ok ? g_variant : 1) {
    case 0: return launch_s<EPI, HD, 0>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 1: return launch_s<EPI, HD, 1>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 2: return launch_s<EPI, HD, 2>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 4: return launch_s<EPI, HD, 4>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 5: return launch_s<EPI, HD, 5>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 6: return launch_s<EPI, HD, 6>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 7: return launch_s<EPI, HD, 7>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 8: return launch_s<EPI, HD, 8>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 9: return launch_s<EPI, HD, 9>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 10: return launch_s<EPI, HD, 10>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
#ifdef ND_GEMM_ABLATION
    case 11: return launch_s<EPI, HD, 11>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 12: return launch_s<EPI, HD, 12>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 13: return launch_s<EPI, HD, 13>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 15: return launch_s<EPI, HD, 15>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 17: return launch_s<EPI, HD, 17>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 18: return launch_s<EPI, HD, 18>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
    case 19: return launch_s<EPI, HD, 19>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
#endif
    default: return launch_s<EPI, HD, 3>(A, B, C, M, N, K, lda, ldb, ldc, ep, s);
  }
}

bool shapes_ok(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc) {
  // byte offsets of one operand tile stay 32-bit (per-lane DMA offsets)
  return M > 0 && N > 0 && K > 0 && K % TK == 0 && N % 4 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0 &&
         lda >= K && ldb >= K && (int64_t)TM * lda * 2 < (1ll << 31) && (int64_t)TN * ldb * 2 < (1ll << 31);
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
ND_API int nd_gemm_set_variant(int v) {
  const int old = g_variant;
  if ((v >= 0 && v <= 10) || (v > 10 && v < 20)) g_variant = v;
  return old;
}

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
