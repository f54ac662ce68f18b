// Projection GEMM, one wave per SIMD (round 4): C[M, N] = A[M, K] . B[N, K]^T, bf16 in, fp32 accumulate.
//
// Why (profiles/r4_hipblaslt_kloop.md): the disassembly of the hipBLASLt kernel that won the plain
// Llama products in round 3 (Custom_Cijk_Alik_Bljk_..._SK3_MT256x256x64_MI16x16x1, torch's bundled
// TensileLibrary_BB_BB_HA_Bias_SAV_..._gfx950.co) is NOT a ping-pong pair: 4 waves, ONE wave per SIMD,
// 128 x 128 outputs per wave (8 x 8 v_mfma_f32_16x16x32_bf16 accumulators = all 256 AGPRs), and a
// single continuous MFMA stream of 128 MFMAs per 64-deep K-tile into which that same wave weaves its
// 32 ds_read_b128 fragment reads, its 16 LDS-DMA pieces (8 rows x 128 B: whole cache lines) and its
// barriers.  Per SIMD that is 32 fragment reads per K-tile instead of the ping-pong pair's 48.
//
// This kernel is that structure, written for our layouts and epilogues:
//
//   * 256 threads; wave w: rows 128 (w >> 1) .., columns 128 (w & 1) .. of the 256 x 256 tile.
//   * LDS: two K-tile buffers of [A 256 rows x 128 B | B 256 rows x 128 B], 16-B chunk index XOR
//     (row >> 1) & 7 (on the DMA source address -- LDS-DMA writes lane-linear -- and on the reads).
//     Every DMA piece is 8 whole 128-B rows: a k-split into 64-B half rows measured 30 % slower (twice
//     the cache-line requests per byte; session r4c ablations, profiles/r4_gemm_w128.md).
//   * Each K-tile i (buffer i & 1) is two PHASES of 64 MFMAs:
//
//       phase 1:  MFMAs on F0 (k-step 0 of i, in registers)
//                 reads F1 <- A k-step 1 of i, lgkmcnt(0), BARRIER (A half of buffer i & 1 free),
//                 reads F1 <- B k-step 1 of i, DMA A of tile i + 2 -> buffer i & 1
//                 then lgkmcnt(0), vmcnt(8): all of tile i + 1 has landed
//       phase 2:  BARRIER (B half free; tile i + 1 visible), MFMAs on F1
//                 DMA B of tile i + 2 -> buffer i & 1 (first half), reads F0 <- k-step 0 of i + 1
//
//     Two barriers per K-tile, each placed between MFMAs; the only vmcnt wait leaves the next
//     tile's A pieces in flight.  A DMA piece has 2-2.5 phases to land.
//   * Persistent grid (one workgroup per CU, XCD-remapped tile walk with GM m-panel groups, as
//     gemm_pp).  OVL: a tile's epilogue is woven into its last phase (row block a - 1 stored 5 MFMAs
//     after its last one), else it runs between the tiles.
//   * B rows are stored PERMUTED in LDS (DMA source rows; reads stay natural) so that each lane's
//     accumulators of column blocks 2p, 2p + 1 are 8 CONSECUTIVE output columns: one 16-B store per
//     (row block, block pair), no cross-lane shuffle.
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
constexpr uint32_t BUFB0 = 2 * 256 * 128;  // one K-tile buffer (A + B, 64 KiB) without padding
constexpr int LGKM0 = 0xC07F;        // s_waitcnt lgkmcnt(0), vmcnt / expcnt at their maxima

enum : int { W_STORE = 0 };

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// one LDS-DMA wave-instruction: 64 lanes x 16 B from descriptor r at per-lane byte offset voff to LDS
// [lds, lds + 1 KiB); lanes past the descriptor's record count read nothing
__device__ __forceinline__ void dma(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds) : "memory");
}
// m0 set one MFMA ahead of its piece (nothing else in these kernels reads m0), then the bare load
__device__ __forceinline__ void set_m0(uint32_t lds) { asm volatile("s_mov_b32 m0, %0" ::"s"(lds) : "memory"); }
__device__ __forceinline__ void dma_go(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(r) : "memory");
}
// FLAT-global form of the piece (saddr + 32-bit voffset, no range check): ABL 4096 probe only
__device__ __forceinline__ void gdma_go(const void* sbase, uint32_t voff) {
  asm volatile("global_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase) : "memory");
}
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}
template <int N> __device__ __forceinline__ void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }
template <int ABL, int N> __device__ __forceinline__ void vmwait_l() {
  if constexpr ((ABL & 16) == 0) vmwait<N>();
}
// MFMAs as inline asm on accumulators pinned to AGPRs with a TIED operand ("+a"): the zero-input
// form of a tile's first k-step then overwrites exactly the registers the previous tile's epilogue has
// just read (a free "=a" result lets the register allocator park the whole old tile in VGPRs and
// spill).  The compiler sees no MFMA, so the code that reads an accumulator after its last MFMA
// waits for the result itself (drain(), or 5 MFMAs in between).
__device__ __forceinline__ void mma(const bf16x8& a, const bf16x8& b, f32x4& c) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mma0(const bf16x8& a, const bf16x8& b, f32x4& c) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void drain() { asm volatile("s_nop 15\n\ts_nop 3" ::: "memory"); }

// stores per wave per tile (8 row blocks x 4 column pairs)
constexpr int NST = 32;
// phase slots of the A DMA pieces (phase 1, after the A barrier) and of the B pieces (phase 2)
// (every covered read is retired 8+ MFMAs after its issue: an lgkmcnt right behind a read stalls the
// lone wave for the read's latency)
__host__ __device__ constexpr bool a_rd1_slot(int s) { return s >= 1 && s <= 15 && (s - 1) % 2 == 0; }   // A k-step 1
constexpr int A_BAR = 23;                                                                             // A free
__host__ __device__ constexpr bool a_dma_slot(int s) { return s >= 24 && (s - 24) % 5 == 0 && s <= 59; }
__host__ __device__ constexpr bool b_rd1_slot(int s) { return s >= 26 && s <= 47 && (s - 26) % 3 == 0; }  // B k-step 1
// phase 2: the B pieces early (they have the rest of this phase and the next one to land)
__host__ __device__ constexpr bool b_dma_slot(int s) { return s >= 3 && s <= 31 && (s - 3) % 4 == 0; }
constexpr int B_DMA_LAST = 31;
// epilogue stores issued after the last B piece of a LAST phase (epi(a - 1) at slot 8 a + 4, epi(7) after)
__host__ __device__ constexpr int nst_tail() {
  int n = 4;
  for (int a = 1; a < 8; ++a) n += (8 * a + 4 > B_DMA_LAST) ? 4 : 0;
  return n;
}

// ABL: ablation builds for profiling only (WRONG results): 1 no LDS-DMA in the phases, 2 no fragment
// reads in the phases, 4 no barriers in the phases, 8 no epilogue stores, 16 no vmcnt waits in the loop;
// 4096: the loop's pieces as FLAT-global LDS loads (no range check: exact-multiple shapes only)
// VB (round 6, verdict r5 item 4, A/B): the B operand staged through VGPRs instead of LDS-DMA -- phase 2 of
// iteration i issues the 8 B pieces of tile i + 2 as plain buffer_load_dwordx4 into 32 VGPRs (same source
// offsets, same slots), phase 1 of iteration i + 1 writes them lane-linear into the B half of buffer
// (i + 2) & 1 with ds_write_b128 at slots 8-22, before that phase's A pieces (so the compiler's own wait for
// the loads counts no asm piece younger than them); the end-of-phase lgkmcnt(0) and the phase-2 barrier make
// them visible exactly as the DMA pieces were.  Only the A operand stays DMA-fed.
template <int EPI, int STP, bool OVL, int ABL = 0, bool VB = false>
__global__ void __launch_bounds__(256, 1) gemm_w128_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                           bf16_t* __restrict__ C, int M, int N, int K, int64_t lda,
                                                           int64_t ldb, int64_t ldc, int GM) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // LDS layout: 32-row blocks (4 KiB: one DMA piece per wave) at a stride PS (hipBLASLt's 64-B pad
  // per block measured +-0: r4_gemm_w128.md)
  constexpr uint32_t PS = 4096u;
  constexpr uint32_t OPB = 8 * PS, BUFB = 2 * OPB;
  const int tn = (N + TN - 1) / TN, tmn = (M + TM - 1) / TM, tiles = tmn * tn;
  const int G = gridDim.x;  // <= tiles (host)
  const int first = xcd_remap(blockIdx.x, G);
  const int my_tiles = (tiles - 1 - first) / G + 1;
  const int nk = K / TK;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);

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

  // ---- LDS-DMA: piece j (0..7) of an operand = LDS rows 8 (w + 4 j) .. + 7 (1 KiB); lane -> LDS row
  // l >> 3, physical chunk l & 7 (lane-linear), which holds logical chunk (l & 7) ^ ((row >> 1) & 7).
  // A: LDS row = tile row.  B: LDS row j holds tile column g(j) (the permutation above).
  uint32_t voa[8], vob[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int row = 8 * (w + 4 * j) + (lane >> 3);
    const int lch = (lane & 7) ^ ((row >> 1) & 7);
    const int jj = row & 127, blk = jj >> 4, i = jj & 15;
    const int gcol = (row & 128) + 32 * (blk >> 1) + 8 * (i >> 2) + 4 * (blk & 1) + (i & 3);
    voa[j] = (uint32_t)(((int64_t)row * lda + lch * 8) * 2);
    vob[j] = (uint32_t)(((int64_t)gcol * ldb + lch * 8) * 2);
  }
  struct Pos { int lt, kt, m0, n0; };
  auto pos_init = [&](Pos& p, int s) __attribute__((always_inline)) {
    p.lt = s / nk;
    p.kt = s - p.lt * nk;
    if (p.lt < my_tiles) coords(first + p.lt * G, p.m0, p.n0);
  };
  auto pos_next = [&](Pos& p) __attribute__((always_inline)) {
    if (++p.kt == nk) {
      p.kt = 0;
      ++p.lt;
      if (p.lt < my_tiles) coords(first + p.lt * G, p.m0, p.n0);
    }
  };
  // descriptors of K-tile p (zero records past the stream's end: the pieces are still issued --
  // constant vmcnt counts -- but read nothing)
  auto rs_a = [&](const Pos& p) __attribute__((always_inline)) {
    const int64_t e0 = (int64_t)p.m0 * lda + (int64_t)p.kt * TK;
    const int64_t lim = (int64_t)M * lda - e0;
    const bool ok = p.lt < my_tiles && lim > 0;
    return rsrc(A + (ok ? e0 : 0), ok ? (uint32_t)(lim < 0x3fffffff ? lim * 2 : 0x7ffffffe) : 0u);
  };
  auto rs_b = [&](const Pos& p) __attribute__((always_inline)) {
    const int64_t e0 = (int64_t)p.n0 * ldb + (int64_t)p.kt * TK;
    const int64_t lim = (int64_t)N * ldb - e0;
    const bool ok = p.lt < my_tiles && lim > 0;
    return rsrc(B + (ok ? e0 : 0), ok ? (uint32_t)(lim < 0x3fffffff ? lim * 2 : 0x7ffffffe) : 0u);
  };
  auto stage_all = [&](const Pos& p, int s) __attribute__((always_inline)) {
    const uint32_t d = lds0 + (uint32_t)(s & 1) * BUFB + (uint32_t)w * 1024u;
    const auto ra = rs_a(p), rb = rs_b(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) dma(ra, voa[j], d + (uint32_t)j * PS);
#pragma unroll
    for (int j = 0; j < 8; ++j) dma(rb, vob[j], d + OPB + (uint32_t)j * PS);
  };

  // ---- fragment reads: A block a = LDS rows 128 wm + 16 a + r16, B block b = LDS rows 128 wn + 16 b + r16;
  // k-step ks: logical chunk 4 ks + q, physical ^ ((row >> 1) & 7) = ^ ((r16 >> 1) & 7)
  const int r16 = lane & 15, q = lane >> 4;
  uint32_t fa_off[2], fb_off[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const uint32_t o = (uint32_t)(r16 * 128 + (((4 * ks + q) ^ ((r16 >> 1) & 7)) << 4));
    fa_off[ks] = o + (uint32_t)wm * 4u * PS;
    fb_off[ks] = o + OPB + (uint32_t)wn * 4u * PS;
  }
  // 16-row block a: 32-row block a >> 1, half a & 1
  auto rd_a = [&](uint32_t base, int ks, int a, bf16x8 (&fa)[8]) __attribute__((always_inline)) {
    fa[a] = *reinterpret_cast<const bf16x8*>(smem + base + fa_off[ks] + (a >> 1) * PS + (a & 1) * 2048);
  };
  auto rd_b = [&](uint32_t base, int ks, int b, bf16x8 (&fb)[8]) __attribute__((always_inline)) {
    fb[b] = *reinterpret_cast<const bf16x8*>(smem + base + fb_off[ks] + (b >> 1) * PS + (b & 1) * 2048);
  };

  f32x4 acc[8][8];
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  int pm0 = 0, pn0 = 0;  // tile of the accumulators (for its epilogue)
  u32x4 sb[8];           // VB: the B pieces of tile i + 2 between their load (phase 2) and ds_write (phase 1)
  bool have_sb = false;

  // ---- epilogue of the 16-row block a of the tile (m0, n0): lane row r16, columns 8 q + 0..7 of each
  // 32-column block pair -> one 16-B store per pair; rows past M drop through the descriptor, columns
  // past N through an offset sentinel
  auto epi = [&](int a, int m0, int n0) __attribute__((always_inline)) {
    const int rows = M - m0 < TM ? M - m0 : TM;
    const auto cr = rsrc(C + (int64_t)m0 * ldc, (uint32_t)((int64_t)rows * ldc * 2));
    const int lrow = 128 * wm + 16 * a + r16;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      // the accumulators reach VGPRs HERE, one v_accvgpr_read per element from an AGPR operand:
      // left to itself the register allocator hoists all 256 AGPR reads to the epilogue's start
      f32x4 x, y;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(x[r]) : "a"(acc[a][2 * p][r]));
        asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(y[r]) : "a"(acc[a][2 * p + 1][r]));
      }
      const u32x4 d = u32x4{pack2(x[0], x[1]), pack2(x[2], x[3]), pack2(y[0], y[1]), pack2(y[2], y[3])};
      const int col = n0 + 128 * wn + 32 * p + 8 * q;
      const uint32_t off = col < N ? (uint32_t)(((int64_t)lrow * ldc + col) * 2) : 0x80000000u;
      if constexpr ((ABL & 8) != 0) asm volatile("" ::"v"(d), "v"(off));
      else __builtin_amdgcn_raw_buffer_store_b128(d, cr, off, 0, STP);
    }
  };

  // ---- phase 1 of K-tile (buffer cur): 64 MFMAs on F0; F1 <- k-step 1 of cur (A reads, barrier, B
  // reads); DMA A of tile i + 2 into cur after the barrier.  hook: the scalar work for phase 2
  // (descriptors, coordinates) between the MFMAs
  const bf16_t* gpa = A;  // ABL 4096 probe: FLAT-global piece base pointers of K-tile i + 2
  const bf16_t* gpb = B;
  auto phase1 = [&](auto FIRST, uint32_t cur, __amdgpu_buffer_rsrc_t dra, uint32_t dlds, auto&& hook)
      __attribute__((always_inline)) {
    constexpr bool F = decltype(FIRST)::value;
    const uint32_t nxt = BUFB - cur;  // VB: the buffer of tile i + 2 (= i & 1 = the other one)
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      const int a = s >> 3, b = s & 7;
      if constexpr (F) mma0(fb0[b], fa0[a], acc[a][b]);
      else mma(fb0[b], fa0[a], acc[a][b]);
      if constexpr (VB) {
        if (s >= 8 && s <= 22 && (s & 1) == 0 && have_sb)
          *reinterpret_cast<u32x4*>(smem + nxt + (uint32_t)w * 1024u + OPB + (uint32_t)((s - 8) / 2) * PS +
                                    (uint32_t)lane * 16u) = sb[(s - 8) / 2];
      }
      if (!(ABL & 2)) {
        if (a_rd1_slot(s)) rd_a(cur, 1, (s - 1) / 2, fa1);
        if (b_rd1_slot(s)) rd_b(cur, 1, (s - 26) / 3, fb1);
      }
      if (s == A_BAR) {  // every wave's A k-step-1 reads retired -> the A half of cur is free
        __builtin_amdgcn_s_waitcnt(LGKM0);
        if (!(ABL & 4)) bar();
      }
      if (a_dma_slot(s) && !(ABL & 1)) {
        if constexpr ((ABL & 4096) != 0) gdma_go(gpa, voa[(s - 24) / 5]);
        else dma_go(dra, voa[(s - 24) / 5]);
      }
      // m0 for the next slot's piece, one MFMA ahead (the bare load then issues without a wait state)
      if (a_dma_slot(s + 1) && !(ABL & 1)) set_m0(dlds + (uint32_t)((s + 1 - 24) / 5) * PS);
      if (s == 40) hook();
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // ---- phase 2: barrier (the B half of cur free; tile i + 1 landed and visible); 64 MFMAs on F1;
  // F0 <- k-step 0 of tile i + 1 (buffer nxt); DMA B of tile i + 2 into cur.  LAST: the tile's epilogue
  // woven in (row block a - 1 five MFMAs after its last one)
  auto phase2 = [&](auto LAST, uint32_t nxt, __amdgpu_buffer_rsrc_t drb, uint32_t dlds, auto&& hook)
      __attribute__((always_inline)) {
    constexpr bool L = decltype(LAST)::value;
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      const int a = s >> 3, b = s & 7;
      mma(fb1[b], fa1[a], acc[a][b]);
      if (s == 1 && !(ABL & 4)) bar();
      if (!(ABL & 2) && s >= 2 && s <= 47 && (s - 2) % 3 == 0) {
        const int r = (s - 2) / 3;
        if (r < 8) rd_a(nxt, 0, r, fa0);
        else rd_b(nxt, 0, r - 8, fb0);
      }
      if (b_dma_slot(s) && !(ABL & 1)) {
        if constexpr (VB) sb[(s - 3) / 4] = __builtin_amdgcn_raw_buffer_load_b128(drb, vob[(s - 3) / 4], 0, 0);
        else if constexpr ((ABL & 4096) != 0) gdma_go(gpb, vob[(s - 3) / 4]);
        else dma_go(drb, vob[(s - 3) / 4]);
      }
      if (!VB && b_dma_slot(s + 1) && !(ABL & 1)) set_m0(dlds + OPB + (uint32_t)((s + 1 - 3) / 4) * PS);
      if (s == 30) hook();
      if constexpr (L) {
        if (b == 4 && a > 0) epi(a - 1, pm0, pn0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (L) {
      drain();
      epi(7, pm0, pn0);
    }
    if constexpr (VB) have_sb = true;
  };

  // ---- prologue: tiles 0 and 1 staged, tile 0 landed, its k-step 0 in F0
  {
    Pos p;
    pos_init(p, 0);
    stage_all(p, 0);
    pos_init(p, 1);
    stage_all(p, 1);
  }
  vmwait<16>();
  bar();
#pragma unroll
  for (int a = 0; a < 8; ++a) rd_a(0, 0, a, fa0);
#pragma unroll
  for (int b = 0; b < 8; ++b) rd_b(0, 0, b, fb0);
  __builtin_amdgcn_s_waitcnt(LGKM0);

  Pos p2;  // K-tile i + 2: the DMA target of iteration i
  pos_init(p2, 2);
  __amdgpu_buffer_rsrc_t dA = rs_a(p2);
  if constexpr ((ABL & 4096) != 0) gpa = A + ((p2.lt < my_tiles) ? (int64_t)p2.m0 * lda + (int64_t)p2.kt * TK : 0);
  constexpr int NST_TAIL = nst_tail();
  // FIRST: the tile's first K-tile (zero-input MFMAs); LAST: its last, with the epilogue woven into its
  // second phase (OVL).  after_epi: 1 the previous iteration was a LAST one, 2 the between-tile
  // epilogue preceded -- its stores are younger than the pieces the phase-1 wait retires
  auto iteration = [&](auto FIRST, auto LAST, int i, int after_epi) __attribute__((always_inline)) {
    const uint32_t cur = (uint32_t)(i & 1) * BUFB, nxt = (uint32_t)((i + 1) & 1) * BUFB;
    const uint32_t dlds = lds0 + cur + (uint32_t)w * 1024u;
    __amdgpu_buffer_rsrc_t dB;
    phase1(FIRST, cur, dA, dlds, [&]() __attribute__((always_inline)) {
      dB = rs_b(p2);
      if constexpr ((ABL & 4096) != 0) gpb = B + ((p2.lt < my_tiles) ? (int64_t)p2.n0 * ldb + (int64_t)p2.kt * TK : 0);
      if constexpr (decltype(FIRST)::value) coords(first + (i / nk) * G, pm0, pn0);  // this tile's epilogue
    });
    __builtin_amdgcn_s_waitcnt(LGKM0);
    // tile i + 1 landed: its A pieces came in iteration i - 1's phase 1, its B pieces in its phase 2;
    // younger: this phase's A pieces of tile i + 2, and any epilogue stores after i + 1's last B piece
    if (after_epi == 1) vmwait_l<ABL, 8 + NST_TAIL>();
    else if (after_epi == 2) vmwait_l<ABL, 8 + NST>();
    else vmwait_l<ABL, 8>();
    phase2(LAST, nxt, dB, dlds, [&]() __attribute__((always_inline)) {
      pos_next(p2);
      dA = rs_a(p2);
      if constexpr ((ABL & 4096) != 0) gpa = A + ((p2.lt < my_tiles) ? (int64_t)p2.m0 * lda + (int64_t)p2.kt * TK : 0);
    });
    __builtin_amdgcn_s_waitcnt(LGKM0);
  };
  auto epilogue_all = [&]() __attribute__((always_inline)) {
    drain();
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      epi(a, pm0, pn0);
      __builtin_amdgcn_sched_barrier(0);  // one row block at a time: bounded epilogue registers
    }
  };
  const std::false_type NO;
  const std::true_type YES;
  if constexpr (OVL) {
    // nk >= 2 (host): every tile = FIRST, plain K-tiles, LAST with the epilogue inside its second phase
    for (int lt = 0, i = 0; lt < my_tiles; ++lt) {
      iteration(YES, NO, i++, lt > 0 ? 1 : 0);
      for (int kt = 1; kt < nk - 1; ++kt) iteration(NO, NO, i++, 0);
      iteration(NO, YES, i++, 0);
    }
  } else {
    for (int lt = 0, i = 0; lt < my_tiles; ++lt) {
      iteration(YES, NO, i++, lt > 0 ? 2 : 0);
      for (int kt = 1; kt < nk; ++kt) iteration(NO, NO, i++, 0);
      // the tile's epilogue between the tiles (matrix pipe idle; the next tile's DMA is in flight)
      epilogue_all();
    }
  }
  vmwait<0>();  // trailing zero-record DMA pieces: retired before the workgroup's LDS is released
}

int g_w128_group_m = [] {
  const char* e = getenv("ND_GEMM_W128_GM");
  return e ? atoi(e) : 4;
}();

int num_cus_w128() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) return 256;
    return v;
  }();
  return n;
}

int g_w128_nt = 1;   // non-temporal C stores
int g_w128_ovl = 1;  // epilogue woven into each tile's last phase (0: between the tiles)
int g_w128_abl = 0;  // ablation variants (profiling only; -DND_ABLATION builds): nd_gemm_w128_set_ablation
int g_w128_vb = [] {  // B operand staged through VGPRs (A/B; nd_gemm_w128_set_vb / ND_GEMM_W128_VB)
  const char* e = getenv("ND_GEMM_W128_VB");
  return e ? atoi(e) : 0;
}();

template <int EPI, int STP, bool OVL, int ABL = 0, bool VB = false>
int launch_w128_v(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
                  hipStream_t s) {
  const size_t lds = 2 * (size_t)BUFB0;  // 128 KiB
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&gemm_w128_kernel<EPI, STP, OVL, ABL, VB>), hipFuncAttributeMaxDynamicSharedMemorySize,
      (int)lds);
  if (attr != hipSuccess) return (int)attr;
  const int tiles = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  const int grid = tiles < num_cus_w128() ? tiles : num_cus_w128();
  hipLaunchKernelGGL((gemm_w128_kernel<EPI, STP, OVL, ABL, VB>), dim3(grid), dim3(256), lds, s, (const bf16_t*)A,
                     (const bf16_t*)B, (bf16_t*)C, M, N, K, lda, ldb, ldc, g_w128_group_m);
  ND_LAUNCH_CHECK();
}

template <int EPI>
int launch_w128(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
                hipStream_t s) {
#ifdef ND_ABLATION
  if constexpr (EPI == W_STORE) {
    switch (g_w128_abl) {
      case 1: return launch_w128_v<EPI, 2, false, 1>(A, B, C, M, N, K, lda, ldb, ldc, s);
      case 2: return launch_w128_v<EPI, 2, false, 2>(A, B, C, M, N, K, lda, ldb, ldc, s);
      case 3: return launch_w128_v<EPI, 2, false, 3>(A, B, C, M, N, K, lda, ldb, ldc, s);
      case 4: return launch_w128_v<EPI, 2, false, 4>(A, B, C, M, N, K, lda, ldb, ldc, s);
      case 8: return launch_w128_v<EPI, 2, false, 8>(A, B, C, M, N, K, lda, ldb, ldc, s);
      case 16: return launch_w128_v<EPI, 2, false, 16>(A, B, C, M, N, K, lda, ldb, ldc, s);
      case 31: return launch_w128_v<EPI, 2, false, 31>(A, B, C, M, N, K, lda, ldb, ldc, s);
      case 4096: return launch_w128_v<EPI, 2, true, 4096>(A, B, C, M, N, K, lda, ldb, ldc, s);  // exact multiples only
      default: break;
    }
  }
#endif
  if (g_w128_vb && g_w128_ovl && g_w128_nt && K >= 2 * TK)
    return launch_w128_v<EPI, 2, true, 0, true>(A, B, C, M, N, K, lda, ldb, ldc, s);
  if (g_w128_ovl && K >= 2 * TK)
    return g_w128_nt ? launch_w128_v<EPI, 2, true>(A, B, C, M, N, K, lda, ldb, ldc, s)
                     : launch_w128_v<EPI, 0, true>(A, B, C, M, N, K, lda, ldb, ldc, s);
  return g_w128_nt ? launch_w128_v<EPI, 2, false>(A, B, C, M, N, K, lda, ldb, ldc, s)
                   : launch_w128_v<EPI, 0, false>(A, B, C, M, N, K, lda, ldb, ldc, s);
}

bool w128_shapes_ok(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc) {
  return M > 0 && N > 0 && K > 0 && K % TK == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 8 == 0 &&
         lda >= K && ldb >= K && (int64_t)TM * lda * 2 < (1ll << 31) && (int64_t)TN * ldb * 2 < (1ll << 31) &&
         (int64_t)TM * ldc * 2 < (1ll << 31);
}
}  // namespace

// C[M, N] = A[M, K] . B[N, K]^T (bf16, fp32 accumulate).  K % 64 == 0, N % 8 == 0, lda / ldb / ldc % 8
// == 0, 16-B aligned base pointers.
ND_API int nd_gemm_w128(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb,
                        int64_t ldc, hipStream_t s) {
  if (!w128_shapes_ok(M, N, K, lda, ldb, ldc)) return (int)hipErrorInvalidValue;
  return launch_w128<W_STORE>(A, B, C, M, N, K, lda, ldb, ldc, s);
}

// the timing ablations (wrong results) exist only in a -DND_ABLATION build: elsewhere this returns -1
ND_API int nd_gemm_w128_set_ablation(int v) {
#ifndef ND_ABLATION
  if (v != 0) return -1;
#endif
  const int old = g_w128_abl;
  g_w128_abl = v;
  return old;
}

// 1: the B operand staged through VGPRs (VB above; the epilogue-in-last-phase, non-temporal form only); returns
// the previous setting
ND_API int nd_gemm_w128_set_vb(int v) {
  const int old = g_w128_vb;
  if (v >= 0) g_w128_vb = v;
  return old;
}

ND_API int nd_gemm_w128_set(int group_m, int nt, int ovl) {
  const int old = g_w128_group_m;
  if (group_m >= 0) g_w128_group_m = group_m;
  if (nt >= 0) g_w128_nt = nt;
  if (ovl >= 0) g_w128_ovl = ovl;
  return old;
}
