// Projection GEMM, one wave per SIMD (round 4): C[M, N] = A[M, K] . B[N, K]^T, bf16 in, fp32 accumulate.
//
// Why (profiles/r4_hipblaslt_kloop.md): the disassembly of the hipBLASLt kernel that won the plain
// Llama products in round 3 (Custom_Cijk_Alik_Bljk_..._SK3_MT256x256x64_MI16x16x1, torch's bundled
// TensileLibrary_BB_BB_HA_Bias_SAV_..._gfx950.co) is NOT a ping-pong pair: 4 waves, ONE wave per SIMD,
// 128 x 128 outputs per wave (8 x 8 v_mfma_f32_16x16x32_bf16 accumulators = all 256 AGPRs), and a
// single continuous MFMA stream of 128 MFMAs per 64-deep K-tile into which that same wave weaves its
// 32 ds_read_b128 fragment reads, its 16 LDS-DMA pieces and three barriers.  Per SIMD that is 32
// fragment reads per K-tile instead of the ping-pong pair's 48 (128 x 128 per wave reuses every
// fragment 8 times instead of 4 / 8), and the matrix pipe never waits for a partner's phase.
//
// This kernel is that structure, written for our layouts and epilogues:
//
//   * 256 threads; wave w: rows 128 (w >> 1) .., columns 128 (w & 1) .. of the 256 x 256 tile.
//   * Each K-tile is two PHASES of 64 MFMAs (k-step 0 = k 0..31, k-step 1 = k 32..63).  LDS holds two
//     K-tile buffers, each split by k-HALF ([h][A 256 rows x 64 B | B 256 rows x 64 B], 16-B chunk
//     index XOR-swizzled by swz4(row >> 2) on the DMA source address and on the reads -- conflict-free
//     for the ds_read_b128 lane groups).  Stream position i (tile, K-tile) lives in buffer i & 1:
//
//       phase 1 of i:  MFMAs on F0 (k-half 0 of i, in registers)
//                      reads  F1 <- k-half 1 of i            DMA  k-half 0 of i + 2 -> buffer i & 1
//                      then   lgkmcnt(0), vmcnt(16): k-half 0 of i + 1 has landed
//       phase 2 of i:  MFMAs on F1
//                      reads  F0 <- k-half 0 of i + 1        DMA  k-half 1 of i + 2 -> buffer i & 1
//                      then   lgkmcnt(0), vmcnt(16): k-half 1 of i + 1 has landed
//
//     ONE barrier per phase, issued after the phase's first two MFMAs (they need only registers), so
//     each DMA has two phases (~2k cycles) to land and every wait is a counted vmcnt.  WAR: a k-half
//     is restaged only after the barrier that follows the lgkmcnt(0) retiring its last reads.
//   * Persistent grid (one workgroup per CU, XCD-remapped tile walk with GM m-panel groups, as
//     gemm_pp).  A tile's epilogue runs inside the next tile's first phase: the 16-row block a of the
//     finished accumulators is converted and stored right before the new tile's zero-input MFMAs
//     overwrite acc[a][*], so its VALU / store issue overlaps the MFMA pipe.
//   * The B fragment rows are permuted (block 2p + e, lane row i -> B row 32 p + 8 (i >> 2) + 4 e +
//     (i & 3)) so that each lane's accumulators of blocks 2p, 2p + 1 are 8 CONSECUTIVE output columns:
//     one 16-B store per (row block, block pair) with no cross-lane shuffle.
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
constexpr uint32_t OPH = 256 * 64;  // one operand's k-half: 256 rows x 64 B (16 KiB)
constexpr uint32_t KH = 2 * OPH;    // A + B of one k-half (32 KiB)
constexpr uint32_t BUFB = 2 * KH;   // one K-tile buffer (64 KiB)
constexpr int LGKM0 = 0xC07F;       // s_waitcnt lgkmcnt(0), vmcnt / expcnt at their maxima

enum : int { W_STORE = 0 };

__device__ __forceinline__ int swz4(int r) { return (0x1320 >> (4 * (r & 3))) & 3; }  // 0, 2, 3, 1

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
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}
template <int N> __device__ __forceinline__ void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }
// MFMAs as inline asm on accumulators pinned to AGPRs with a TIED operand ("+a"): the zero-input
// form of a tile's first k-step then overwrites exactly the registers the previous tile's epilogue has
// just read (a free "=a" result lets the register allocator park the whole old tile in VGPRs and
// spill).  The compiler sees no MFMA, so the code that reads an accumulator after its last MFMA
// waits for the result itself (drain()).
__device__ __forceinline__ void mma(const bf16x8& a, const bf16x8& b, f32x4& c) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mma0(const bf16x8& a, const bf16x8& b, f32x4& c) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void drain() { asm volatile("s_nop 15\n\ts_nop 3" ::: "memory"); }

// stores per wave per tile (8 row blocks x 4 column pairs)
constexpr int NST = 32;

template <int EPI, int STP>
__global__ void __launch_bounds__(256, 1) gemm_w128_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                           bf16_t* __restrict__ C, int M, int N, int K, int64_t lda,
                                                           int64_t ldb, int64_t ldc, int GM) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tn = (N + TN - 1) / TN, tmn = (M + TM - 1) / TM, tiles = tmn * tn;
  const int G = gridDim.x;  // <= tiles (host)
  const int first = xcd_remap(blockIdx.x, G);
  const int my_tiles = (tiles - 1 - first) / G + 1;
  const int nk = K / TK;
  const int total = my_tiles * nk;
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

  // ---- LDS-DMA: piece j (0..3) of an operand's k-half = 16-row block w + 4 j; lane -> row l >> 2,
  // physical chunk l & 3 (lane-linear), which holds logical chunk (l & 3) ^ swz4(row >> 2)
  uint32_t voa[4], vob[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 16 * (w + 4 * j) + (lane >> 2);
    const int lch = (lane & 3) ^ swz4(lane >> 4);
    voa[j] = (uint32_t)(((int64_t)row * lda + lch * 8) * 2);
    vob[j] = (uint32_t)(((int64_t)row * ldb + lch * 8) * 2);
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
  // descriptors of k-half h of stream position p (zero records past the stream's end: the pieces
  // are still issued -- constant vmcnt counts -- but read nothing)
  auto rs_a = [&](const Pos& p, int h) __attribute__((always_inline)) {
    const int64_t e0 = (int64_t)p.m0 * lda + (int64_t)p.kt * TK + h * 32;
    const int64_t lim = (int64_t)M * lda - e0;
    const bool ok = p.lt < my_tiles && lim > 0;
    return rsrc(A + (ok ? e0 : 0), ok ? (uint32_t)(lim < 0x3fffffff ? lim * 2 : 0x7ffffffe) : 0u);
  };
  auto rs_b = [&](const Pos& p, int h) __attribute__((always_inline)) {
    const int64_t e0 = (int64_t)p.n0 * ldb + (int64_t)p.kt * TK + h * 32;
    const int64_t lim = (int64_t)N * ldb - e0;
    const bool ok = p.lt < my_tiles && lim > 0;
    return rsrc(B + (ok ? e0 : 0), ok ? (uint32_t)(lim < 0x3fffffff ? lim * 2 : 0x7ffffffe) : 0u);
  };
  auto stage_all = [&](const Pos& p, int s, int h) __attribute__((always_inline)) {
    const uint32_t d = lds0 + (uint32_t)(s & 1) * BUFB + (uint32_t)h * KH + (uint32_t)w * 1024u;
    const auto ra = rs_a(p, h), rb = rs_b(p, h);
#pragma unroll
    for (int j = 0; j < 4; ++j) dma(ra, voa[j], d + (uint32_t)j * 4096u);
#pragma unroll
    for (int j = 0; j < 4; ++j) dma(rb, vob[j], d + OPH + (uint32_t)j * 4096u);
  };

  // ---- fragment reads (per-lane byte offsets inside one k-half): A block a = rows 128 wm + 16 a + r16,
  // B block 2 p + e = rows 128 wn + 32 p + 8 (r16 >> 2) + 4 e + (r16 & 3); chunk q ^ swz4(row >> 2)
  const int r16 = lane & 15, q = lane >> 4;
  const uint32_t fa_off = (uint32_t)((128 * wm + r16) * 64 + ((q ^ swz4(r16 >> 2)) << 4));
  uint32_t fb_off[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int row = 128 * wn + 8 * (r16 >> 2) + 4 * e + (r16 & 3);
    fb_off[e] = OPH + (uint32_t)(row * 64 + ((q ^ swz4(row >> 2)) << 4));
  }
  auto rd = [&](uint32_t base, int r, bf16x8 (&fa)[8], bf16x8 (&fb)[8]) __attribute__((always_inline)) {
    if (r < 8) {
      fa[r] = *reinterpret_cast<const bf16x8*>(smem + base + fa_off + r * 1024);
    } else {
      const int b = r - 8;
      fb[b] = *reinterpret_cast<const bf16x8*>(smem + base + fb_off[b & 1] + (b >> 1) * 2048);
    }
  };

  f32x4 acc[8][8];
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  // ---- epilogue of the 16-row block a of the tile (m0, n0): lane row r16, columns 8 q + 0..7 of each
  // 32-column block pair -> one 16-B store per pair; rows past M drop through the descriptor, columns
  // past N through an offset sentinel
  auto epi = [&](int a, int m0, int n0) __attribute__((always_inline)) {
    const int rows = M - m0 < TM ? M - m0 : TM;
    const auto cr = rsrc(C + (int64_t)m0 * ldc, (uint32_t)((int64_t)rows * ldc * 2));
    const int lrow = 128 * wm + 16 * a + r16;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      // the accumulators reach VGPRs HERE (an empty asm with a VGPR operand tied to the AGPR value):
      // left to itself the register allocator hoists all 256 AGPR reads to the epilogue's start
      f32x4 x, y;
      asm volatile("" : "=v"(x) : "0"(acc[a][2 * p]));
      asm volatile("" : "=v"(y) : "0"(acc[a][2 * p + 1]));
      const u32x4 d = u32x4{pack2(x[0], x[1]), pack2(x[2], x[3]), pack2(y[0], y[1]), pack2(y[2], y[3])};
      const int col = n0 + 128 * wn + 32 * p + 8 * q;
      const uint32_t off = col < N ? (uint32_t)(((int64_t)lrow * ldc + col) * 2) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(d, cr, off, 0, STP);
    }
  };

  // ---- one phase: 64 MFMAs (row block a = s >> 3, column block b = s & 7) with the phase's 16
  // fragment reads and 8 DMA pieces woven in; the barrier after slot 1.  FIRST: zero-input MFMAs;
  // FAT: the previous tile's epilogue of row block a right before slot 8 a
  auto phase = [&](auto FIRST, auto FAT, bf16x8 (&ua)[8], bf16x8 (&ub)[8], uint32_t rbase, bf16x8 (&ra_)[8],
                   bf16x8 (&rb_)[8], __amdgpu_buffer_rsrc_t dra, __amdgpu_buffer_rsrc_t drb, uint32_t dlds, int pm0,
                   int pn0) __attribute__((always_inline)) {
    constexpr bool F = decltype(FIRST)::value, FT = decltype(FAT)::value;
#pragma unroll
    for (int s = 0; s < 64; ++s) {
      const int a = s >> 3, b = s & 7;
      if constexpr (FT) {
        if (b == 0) {
          epi(a, pm0, pn0);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if constexpr (F) mma0(ub[b], ua[a], acc[a][b]);
      else mma(ub[b], ua[a], acc[a][b]);
      if (s == 1) bar();
      if (s >= 2 && s <= 47 && (s - 2) % 3 == 0) rd(rbase, (s - 2) / 3, ra_, rb_);
      if (s >= 3 && (s - 3) % 8 == 0) {
        const int j = (s - 3) / 8;
        if (j < 4) dma(dra, voa[j], dlds + (uint32_t)j * 4096u);
        else dma(drb, vob[j - 4], dlds + OPH + (uint32_t)(j - 4) * 4096u);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- prologue: stream positions 0 and 1 staged, position 0 landed, its k-half 0 in F0
  {
    Pos p;
    pos_init(p, 0);
    stage_all(p, 0, 0);
    stage_all(p, 0, 1);
    pos_init(p, 1);
    stage_all(p, 1, 0);
    stage_all(p, 1, 1);
  }
  vmwait<16>();
  bar();
#pragma unroll
  for (int r = 0; r < 16; ++r) rd(0, r, fa0, fb0);
  __builtin_amdgcn_s_waitcnt(LGKM0);

  Pos p2;  // stream position i + 2: the DMA target of iteration i
  pos_init(p2, 2);
  int pm0 = 0, pn0 = 0;  // tile of the accumulators (epilogue of the FAT phase)

  auto iteration = [&](auto FIRST, auto FAT, int i) __attribute__((always_inline)) {
    constexpr bool FT = decltype(FAT)::value;
    const uint32_t cur = (uint32_t)(i & 1) * BUFB, nxt = (uint32_t)((i + 1) & 1) * BUFB;
    const uint32_t dlds = lds0 + cur + (uint32_t)w * 1024u;
    int em0 = pm0, en0 = pn0;
    if constexpr (decltype(FIRST)::value) {  // this tile's coordinates, for the next epilogue
      const int lt = i / nk;
      coords(first + lt * G, pm0, pn0);
    }
    // phase 1: F0; reads F1 <- k-half 1 of i; DMA k-half 0 of i + 2
    phase(FIRST, FAT, fa0, fb0, cur + KH, fa1, fb1, rs_a(p2, 0), rs_b(p2, 0), dlds, em0, en0);
    __builtin_amdgcn_s_waitcnt(LGKM0);
    vmwait<FT ? 16 + NST : 16>();
    // phase 2: F1; reads F0 <- k-half 0 of i + 1; DMA k-half 1 of i + 2
    phase(std::false_type{}, std::false_type{}, fa1, fb1, nxt, fa0, fb0, rs_a(p2, 1), rs_b(p2, 1), dlds + KH, 0, 0);
    __builtin_amdgcn_s_waitcnt(LGKM0);
    vmwait<FT ? 16 + NST : 16>();
    pos_next(p2);
  };

  for (int lt = 0, i = 0; lt < my_tiles; ++lt) {
    iteration(std::true_type{}, std::false_type{}, i++);
    for (int kt = 1; kt < nk; ++kt) iteration(std::false_type{}, std::false_type{}, i++);
    // the tile's epilogue (v1: between the tiles, matrix pipe idle; the next tile's DMA is in flight)
    drain();
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      epi(a, pm0, pn0);
      __builtin_amdgcn_sched_barrier(0);  // one row block at a time: bounded epilogue registers
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

int g_w128_nt = 1;  // non-temporal C stores

template <int EPI, int STP>
int launch_w128_v(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
                  hipStream_t s) {
  const size_t lds = 2 * (size_t)BUFB;  // 128 KiB
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_w128_kernel<EPI, STP>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return (int)attr;
  const int tiles = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  const int grid = tiles < num_cus_w128() ? tiles : num_cus_w128();
  hipLaunchKernelGGL((gemm_w128_kernel<EPI, STP>), dim3(grid), dim3(256), lds, s, (const bf16_t*)A, (const bf16_t*)B,
                     (bf16_t*)C, M, N, K, lda, ldb, ldc, g_w128_group_m);
  ND_LAUNCH_CHECK();
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
  return g_w128_nt ? launch_w128_v<W_STORE, 2>(A, B, C, M, N, K, lda, ldb, ldc, s)
                   : launch_w128_v<W_STORE, 0>(A, B, C, M, N, K, lda, ldb, ldc, s);
}

ND_API int nd_gemm_w128_set(int group_m, int nt) {
  const int old = g_w128_group_m;
  if (group_m >= 0) g_w128_group_m = group_m;
  if (nt >= 0) g_w128_nt = nt;
  return old;
}
