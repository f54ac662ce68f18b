// Weight-gradient GEMM for gfx950:  C[M, N] (fp32) += A^T B,  A = dY [K, M], B = X [K, N]  (bf16, row-major)
//
// Why a custom kernel: in the wgrad product the reduction dimension K is the token axis, which is the
// STRIDED axis of both operands as they come out of the forward / backward.  hipBLASLt runs this
// "K-outer" layout at 330-900 TF/s on the Llama-150M shapes (vs 1.1-1.4 PF/s for fwd / dgrad), and
// the tall-skinny shapes (M x N = 1024 x 1024 with K = 32768) give too few output tiles to fill
// 256 CUs.  Here:
//   * both operands are staged through LDS exactly as they sit in memory ([k][m] / [k][n] rows,
//     16-B coalesced global loads) and the MFMA fragments (8 consecutive k of one m / n) are fetched
//     with the gfx950 transposing read ds_read_b64_tr_b16 -- no transpose pass in HBM;
//   * LDS rows are XOR-swizzled ((row & 3) << 2 on the 16-B chunk index) so the four rows one
//     32-lane half reads land in four different quarters of the bank row (conflict-free);
//   * split-K: when the output has few tiles, K is split over S workgroups writing fp32 slabs that a
//     streaming kernel sums into C in a fixed order -- deterministic (no float atomics);
//   * register-staged prefetch of the next 64-deep K tile is issued before the current tile's MFMAs;
//   * XCD-aware block remap so the workgroups sharing an A row-panel run on one XCD's L2.
// Tile: 128 x 128 per 256-thread workgroup (2 x 2 waves of 64 x 64, 2 x 2 v_mfma_f32_32x32x16_bf16).
#include "common.h"
#include <cstdlib>
#include <type_traits>


using namespace nd;

typedef __bf16 bfv8 __attribute__((ext_vector_type(8)));
typedef short sv4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int BM = 128, BN = 128, BK = 64;

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0, 0);
}

__device__ __forceinline__ sv4 tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((sv4 __attribute__((address_space(3)))*)(p));
}

// [BK][128] bf16 tile, 256-B rows, 16-B chunk index XOR (row & 3) << 2.
__device__ __forceinline__ int toff(int row, int col) {
  return row * 128 + (((col >> 3) ^ ((row & 3) << 2)) << 3) + (col & 7);
}

// Fragment with k (tile rows) natural: element j of lane half h = row kbase + 8h + j, column cbase + (lane & 31).
__device__ __forceinline__ bf16x8 frag(const bf16_t* tile, int kbase, int cbase, int g, int i) {
  const int row = kbase + 8 * (g >> 1) + (i >> 2);
  const int col = cbase + 16 * (g & 1) + 4 * (i & 3);
  const sv4 lo = tr_read(&tile[toff(row, col)]);
  const sv4 hi = tr_read(&tile[toff(row + 4, col)]);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

struct TileLoad {
  static constexpr int N = (BK * 16) / 256;  // 16-B chunks per thread (4)
  bf16x8 v[N];
  __device__ __forceinline__ void load(const bf16_t* base, int64_t ld, int k0, int kend, int c0, int cols) {
#pragma unroll
    for (int it = 0; it < N; ++it) {
      const int c = threadIdx.x + it * 256;
      const int row = c >> 4, ch = c & 15;
      const int k = k0 + row, col = c0 + ch * 8;
      if (k < kend && col < cols) v[it] = *reinterpret_cast<const bf16x8*>(base + (int64_t)k * ld + col);
      else v[it] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  __device__ __forceinline__ void store(bf16_t* tile) const {
#pragma unroll
    for (int it = 0; it < N; ++it) {
      const int c = threadIdx.x + it * 256;
      const int row = c >> 4, ch = c & 15;
      *reinterpret_cast<bf16x8*>(&tile[toff(row, ch * 8)]) = v[it];
    }
  }
};

}  // namespace

// grid = tiles * S;  S == 1: C += acc in place;  S > 1: slab[s][M][N] = acc.
__global__ void __launch_bounds__(256, 2) wgrad_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                       float* __restrict__ C, float* __restrict__ slab, int M, int N,
                                                       int K, int64_t lda, int64_t ldb, int64_t ldc, int S, int kchunk) {
  __shared__ __attribute__((aligned(16))) bf16_t As[BK * BM];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[BK * BN];
  const int tn_count = (N + BN - 1) / BN;
  const int tiles = ((M + BM - 1) / BM) * tn_count;
  const int id = xcd_remap(blockIdx.x, tiles * S);
  const int split = id / tiles, tile = id % tiles;  // one XCD: same K range, neighbouring tiles (L2 reuse)
  const int m0 = (tile / tn_count) * BM, n0 = (tile % tn_count) * BN;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15;
  const int wm = w >> 1, wn = w & 1;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};

  TileLoad la, lb;
  la.load(A, lda, kbeg, kend, m0, M);
  lb.load(B, ldb, kbeg, kend, n0, N);
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
    la.store(As);
    lb.store(Bs);
    __syncthreads();
    if (k0 + BK < kend) {
      la.load(A, lda, k0 + BK, kend, m0, M);
      lb.load(B, ldb, k0 + BK, kend, n0, N);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) fa[a] = frag(As, ks * 16, wm * 64 + a * 32, g, i16);
#pragma unroll
      for (int b = 0; b < 2; ++b) fb[b] = frag(Bs, ks * 16, wn * 64 + b * 32, g, i16);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma32(fa[a], fb[b], acc[a][b]);
    }
  }
  // epilogue: row m = m0 + wm*64 + a*32 + (r&3) + 8(r>>2) + 4h ; col n = n0 + wn*64 + b*32 + c32
  float* out = S == 1 ? C : slab + (int64_t)split * M * N;
  const int64_t ldo = S == 1 ? ldc : N;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n = n0 + wn * 64 + b * 32 + c32;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M) {
          float* p = out + (int64_t)m * ldo + n;
          if (S == 1) *p += acc[a][b][r];
          else *p = acc[a][b][r];
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Large-tile variant: 256 x 256 per 512-thread workgroup (8 waves as 2 (M) x 4 (N), 128 x 64 each =
// 4 x 2 MFMA tiles), BK = 32, DOUBLE-BUFFERED LDS with one barrier per K tile:
//   compute(buf[k&1]) | global loads of tile k+2 in flight | write tile k+1 regs -> buf[(k+1)&1] | barrier
// 1.5 transposing LDS reads per MFMA (vs 2 in the 128 x 128 kernel), 16 MFMAs per wave per barrier.
namespace {
constexpr int BM2 = 256, BN2 = 256, BK2 = 32;

// [BK2][256] bf16 tile, 512-B rows: 16-B chunk index XOR ((row & 3) << 2) -> the four rows a 32-lane
// half reads with ds_read_b64_tr_b16 fall in different quarters of the 256-B bank row.
__device__ __forceinline__ int toff2(int row, int col) {
  return row * 256 + (((col >> 3) ^ ((row & 3) << 2)) << 3) + (col & 7);
}

__device__ __forceinline__ bf16x8 frag2(const bf16_t* tile, int kbase, int cbase, int g, int i) {
  const int row = kbase + 8 * (g >> 1) + (i >> 2);
  const int col = cbase + 16 * (g & 1) + 4 * (i & 3);
  const sv4 lo = tr_read(&tile[toff2(row, col)]);
  const sv4 hi = tr_read(&tile[toff2(row + 4, col)]);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

struct TileLoad2 {  // BK2 x 256 bf16 = 1024 16-B chunks over 512 threads
  bf16x8 v[2];
  __device__ __forceinline__ void load(const bf16_t* base, int64_t ld, int k0, int kend, int c0, int cols) {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int c = threadIdx.x + it * 512;
      const int row = c >> 5, ch = c & 31;
      const int k = k0 + row, col = c0 + ch * 8;
      if (k < kend && col < cols) v[it] = *reinterpret_cast<const bf16x8*>(base + (int64_t)k * ld + col);
      else v[it] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  __device__ __forceinline__ void store(bf16_t* tile) const {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int c = threadIdx.x + it * 512;
      const int row = c >> 5, ch = c & 31;
      *reinterpret_cast<bf16x8*>(&tile[toff2(row, ch * 8)]) = v[it];
    }
  }
};
}  // namespace

__global__ void __launch_bounds__(512, 2) wgrad256_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                          float* __restrict__ C, float* __restrict__ slab, int M, int N,
                                                          int K, int64_t lda, int64_t ldb, int64_t ldc, int S,
                                                          int kchunk) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  // buffer b: A at smem + b * BK2 * BM2, B at smem + 2 * BK2 * BM2 + b * BK2 * BN2
  const int tn_count = (N + BN2 - 1) / BN2;
  const int tiles = ((M + BM2 - 1) / BM2) * tn_count;
  const int id = xcd_remap(blockIdx.x, tiles * S);
  const int split = id / tiles, tile = id % tiles;  // one XCD: same K range, neighbouring tiles (L2 reuse)
  const int m0 = (tile / tn_count) * BM2, n0 = (tile % tn_count) * BN2;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15;
  const int wm = w >> 2, wn = w & 3;  // 2 x 4 waves, wave tile 128 (M) x 64 (N)

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};

  const int nk = (kend - kbeg + BK2 - 1) / BK2;
  TileLoad2 la, lb;
  if (nk > 0) {
    la.load(A, lda, kbeg, kend, m0, M);
    lb.load(B, ldb, kbeg, kend, n0, N);
    la.store(smem);
    lb.store(smem + 2 * BK2 * BM2);
  }
  __syncthreads();
  if (nk > 1) {
    la.load(A, lda, kbeg + BK2, kend, m0, M);
    lb.load(B, ldb, kbeg + BK2, kend, n0, N);
  }
  for (int kt = 0; kt < nk; ++kt) {
    const bf16_t* a_t = smem + (kt & 1) * BK2 * BM2;
    const bf16_t* b_t = smem + 2 * BK2 * BM2 + (kt & 1) * BK2 * BN2;
#pragma unroll
    for (int ks = 0; ks < BK2 / 16; ++ks) {
      bf16x8 fb[2];
#pragma unroll
      for (int b = 0; b < 2; ++b) fb[b] = frag2(b_t, ks * 16, wn * 64 + b * 32, g, i16);
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const bf16x8 fa = frag2(a_t, ks * 16, wm * 128 + a * 32, g, i16);
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma32(fa, fb[b], acc[a][b]);
      }
    }
    if (kt + 1 < nk) {
      la.store(smem + ((kt + 1) & 1) * BK2 * BM2);
      lb.store(smem + 2 * BK2 * BM2 + ((kt + 1) & 1) * BK2 * BN2);
    }
    __syncthreads();
    if (kt + 2 < nk) {
      la.load(A, lda, kbeg + (kt + 2) * BK2, kend, m0, M);
      lb.load(B, ldb, kbeg + (kt + 2) * BK2, kend, n0, N);
    }
  }
  float* out = S == 1 ? C : slab + (int64_t)split * M * N;
  const int64_t ldo = S == 1 ? ldc : N;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n = n0 + wn * 64 + b * 32 + c32;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 128 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M) {
          float* p = out + (int64_t)m * ldo + n;
          if (S == 1) *p += acc[a][b][r];
          else *p = acc[a][b][r];
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA variant (the production path): same 256 x 256 / 8-wave / 128 x 64-per-wave geometry, but
// tiles move global -> LDS with global_load_lds_dwordx4 (no VGPR round trip, no ds_write issue cost,
// which bounded the register-staged kernel).  The LDS image is lane-linear per wave-instruction
// (1 KiB = two 512-B rows), so the bank swizzle is applied on the SOURCE address: the lane that
// lands in physical chunk p of row r loads logical chunk p ^ ((r & 3) << 2), and the transposing
// reads use the same involution.  BK = 64, two buffers (128 KiB LDS, one workgroup per CU):
//   barrier | DMA tile k+1 -> buf[(k+1)&1] | 32 MFMAs per wave on buf[k&1] | vmcnt(0)+barrier
// A K-tail tile (rows past kend must read as zero) falls back to register staging with zero fill.
namespace {
constexpr int BK3 = 64;
typedef __attribute__((address_space(3))) void lds_void;

// One 16-B-per-lane LDS-DMA wave-instruction, issued from inline asm so hipcc does not track it:
// otherwise it conservatively waits vmcnt(0) before the first LDS read of the OTHER buffer, which
// serialises the DMA of tile k+1 with the MFMAs of tile k.  The caller owns the vmcnt wait.
// M0 (DMA destination base) is compiler-reserved: saved/restored inside the same statement.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_byte_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_byte_addr)
      : "memory");
}

// saddr form: 64-bit uniform base in SGPRs + 32-bit per-lane byte offset (no per-lane 64-bit math).
__device__ __forceinline__ void glds16s(const void* sbase, uint32_t voff, uint32_t lds_byte_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds_byte_addr)
      : "memory");
}

// Per-lane DMA source offsets of a 64 x 256 operand tile, computed once per kernel: the tile at
// K offset k0 is then 4 wave-instructions from the uniform base  base + (k0 + 16 it) * ld,
// with the same per-lane byte offset (row-in-pair * ld + swizzled, clamped column) * 2.
struct DmaPlan {
  uint32_t voff;   // per-lane byte offset inside a row pair
  uint32_t lds0;   // wave's first 1-KiB destination (pair w) relative to the tile base
  __device__ __forceinline__ void init(int64_t ld, int c0, int cols) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int rp = lane >> 5;                       // row inside the pair (rows 2 pair + rp)
    const int p = lane & 31;
    // row & 3 == (2 w + rp) & 3 for every it (rows advance by 16)
    const int c = p ^ (((2 * w + rp) & 3) << 2);
    int col = c0 + c * 8;
    col = col < cols ? col : cols - 8;
    voff = (uint32_t)(((int64_t)rp * ld + col) * 2);
    lds0 = (uint32_t)(w * 1024);
  }
  // rows 2w + 16 it + {0,1} of tile k0 -> LDS tile at byte address tile_addr
  __device__ __forceinline__ void issue(const bf16_t* base, int64_t ld, int k0, uint32_t tile_addr) const {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const bf16_t* sb = base + (int64_t)(k0 + 2 * w + 16 * it) * ld;
      glds16s(sb, voff, tile_addr + (uint32_t)((w + 8 * it) * 1024));
    }
  }
};

__device__ __forceinline__ void dma_tile(bf16_t* tile, const bf16_t* base, int64_t ld, int k0, int c0, int cols) {
  // 64 rows x 512 B = 32 wave-instructions of 1 KiB; wave w issues rows (2i, 2i+1) for i = w, w+8, w+16, w+24
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t tile_addr = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf16_t*)tile);
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int pair = w + 8 * it;
    const int row = 2 * pair + (lane >> 5);
    const int p = lane & 31;                       // physical chunk written by this lane
    const int c = p ^ ((row & 3) << 2);            // logical chunk it must carry
    int col = c0 + c * 8;
    col = col < cols ? col : cols - 8;             // clamp: tail columns only feed masked outputs
    const bf16_t* src = base + (int64_t)(k0 + row) * ld + col;
    glds16(src, __builtin_amdgcn_readfirstlane(tile_addr + pair * 1024));
  }
}

__device__ __forceinline__ void reg_tile(bf16_t* tile, const bf16_t* base, int64_t ld, int k0, int kend, int c0,
                                         int cols) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int c = threadIdx.x + it * 512;
    const int row = c >> 5, ch = c & 31;
    const int k = k0 + row, col = c0 + ch * 8;
    bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (k < kend && col < cols) v = *reinterpret_cast<const bf16x8*>(base + (int64_t)k * ld + col);
    *reinterpret_cast<bf16x8*>(&tile[toff2(row, ch * 8)]) = v;
  }
}
}  // namespace

template <bool SCHED, bool NODMA = false>  // NODMA: diagnostic only (skips the loads; garbage result)
__global__ void __launch_bounds__(512, 2) wgrad_dma_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                           float* __restrict__ C, float* __restrict__ slab, int M,
                                                           int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int S,
                                                           int kchunk) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  constexpr int TA = BK3 * BM2, TB = BK3 * BN2;  // elements per operand tile
  const int tn_count = (N + BN2 - 1) / BN2;
  const int tiles = ((M + BM2 - 1) / BM2) * tn_count;
  const int id = xcd_remap(blockIdx.x, tiles * S);
  const int split = id / tiles, tile = id % tiles;  // one XCD: same K range, neighbouring tiles (L2 reuse)
  const int m0 = (tile / tn_count) * BM2, n0 = (tile % tn_count) * BN2;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15;
  const int wm = w >> 2, wn = w & 3;

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};

  const int nk = kend > kbeg ? (kend - kbeg + BK3 - 1) / BK3 : 0;
  DmaPlan pa, pb;
  pa.init(lda, m0, M);
  pb.init(ldb, n0, N);
  const uint32_t lds_base = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf16_t*)smem);
  auto stage = [&](int kt) {
    if (NODMA) return;
    bf16_t* ta = smem + (kt & 1) * (TA + TB);
    bf16_t* tb = ta + TA;
    const int k0 = kbeg + kt * BK3;
    if (k0 + BK3 <= kend) {
      const uint32_t la = lds_base + (uint32_t)((kt & 1) * (TA + TB) * 2);
      pa.issue(A, lda, k0, la);
      pb.issue(B, ldb, k0, la + TA * 2);
    } else {
      reg_tile(ta, A, lda, k0, kend, m0, M);
      reg_tile(tb, B, ldb, k0, kend, n0, N);
    }
  };
  if (nk > 0) stage(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) stage(kt + 1);
    const bf16_t* a_t = smem + (kt & 1) * (TA + TB);
    const bf16_t* b_t = a_t + TA;
    // fragments of k-step ks+1 are read while the 8 MFMAs of k-step ks run (register double buffer)
    bf16x8 fa[2][4], fb[2][2];
#pragma unroll
    for (int b = 0; b < 2; ++b) fb[0][b] = frag2(b_t, 0, wn * 64 + b * 32, g, i16);
#pragma unroll
    for (int a = 0; a < 4; ++a) fa[0][a] = frag2(a_t, 0, wm * 128 + a * 32, g, i16);
#pragma unroll
    for (int ks = 0; ks < BK3 / 16; ++ks) {
      const int cur = ks & 1, nxt = cur ^ 1;
      if (ks + 1 < BK3 / 16) {
#pragma unroll
        for (int b = 0; b < 2; ++b) fb[nxt][b] = frag2(b_t, (ks + 1) * 16, wn * 64 + b * 32, g, i16);
#pragma unroll
        for (int a = 0; a < 4; ++a) fa[nxt][a] = frag2(a_t, (ks + 1) * 16, wm * 128 + a * 32, g, i16);
      }
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma32(fa[cur][a], fb[cur][b], acc[a][b]);
      if (SCHED && ks + 1 < BK3 / 16) {
        // interleave the 12 transposing reads of k-step ks+1 between the 8 MFMAs of k-step ks
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // 2 DS reads
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of tile kt+1 has landed
    __syncthreads();                                  // ... everyone's, and buf[kt&1] is free again
  }
  float* out = S == 1 ? C : slab + (int64_t)split * M * N;
  const int64_t ldo = S == 1 ? ldc : N;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n = n0 + wn * 64 + b * 32 + c32;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 128 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M) {
          float* p = out + (int64_t)m * ldo + n;
          if (S == 1) *p += acc[a][b][r];
          else *p = acc[a][b][r];
        }
      }
    }
}



// ---------------------------------------------------------------------------------------------
// 16x16x32 variant of the LDS-DMA kernel.  On random data the chip holds a higher clock on
// v_mfma_f32_16x16x32_bf16 loops than on 32x32x16 ones at equal cycles per FLOP (MI355X_MICROARCH
// 'clock', item 7), so the same 256 x 256 tile is computed as 8 x 4 16x16 tiles per wave.
// A 16x16x32 fragment needs k rows 0-3 / 8-11 in one 32-lane half, so the swizzle also folds row bit
// 3 into chunk bit 1:  phys_chunk = chunk ^ ((row & 3) << 2 | ((row >> 3) & 1) << 1)  (conflict-free
// for the transposing reads; applied on the DMA source address as before).
namespace {
__device__ __forceinline__ int swz16(int row) { return ((row & 3) << 2) | (((row >> 3) & 1) << 1); }
__device__ __forceinline__ int toff16(int row, int col) {
  return row * 256 + (((col >> 3) ^ swz16(row)) << 3) + (col & 7);
}
// lane l: column cbase + (l & 15), k rows kbase + 8 (l >> 4) + 0..7
__device__ __forceinline__ bf16x8 frag16(const bf16_t* tile, int kbase, int cbase, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = kbase + 8 * g + (i >> 2);
  const int col = cbase + 4 * (i & 3);
  const sv4 lo = tr_read(&tile[toff16(row, col)]);
  const sv4 hi = tr_read(&tile[toff16(row + 4, col)]);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0, 0);
}
__device__ __forceinline__ void dma_tile16(bf16_t* tile, const bf16_t* base, int64_t ld, int k0, int c0, int cols) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t tile_addr = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf16_t*)tile);
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int pair = w + 8 * it;
    const int row = 2 * pair + (lane >> 5);
    const int c = (lane & 31) ^ swz16(row);
    int col = c0 + c * 8;
    col = col < cols ? col : cols - 8;
    glds16(base + (int64_t)(k0 + row) * ld + col, __builtin_amdgcn_readfirstlane(tile_addr + pair * 1024));
  }
}
__device__ __forceinline__ void reg_tile16(bf16_t* tile, const bf16_t* base, int64_t ld, int k0, int kend, int c0,
                                           int cols) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int c = threadIdx.x + it * 512;
    const int row = c >> 5, ch = c & 31;
    const int k = k0 + row, col = c0 + ch * 8;
    bf16x8 v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (k < kend && col < cols) v = *reinterpret_cast<const bf16x8*>(base + (int64_t)k * ld + col);
    *reinterpret_cast<bf16x8*>(&tile[toff16(row, ch * 8)]) = v;
  }
}
}  // namespace

__global__ void __launch_bounds__(512, 2) wgrad_m16_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                           float* __restrict__ C, float* __restrict__ slab, int M,
                                                           int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int S,
                                                           int kchunk) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  constexpr int TA = BK3 * BM2, TB = BK3 * BN2;
  const int tn_count = (N + BN2 - 1) / BN2;
  const int tiles = ((M + BM2 - 1) / BM2) * tn_count;
  const int id = xcd_remap(blockIdx.x, tiles * S);
  const int split = id / tiles, tile = id % tiles;  // one XCD: same K range, neighbouring tiles (L2 reuse)
  const int m0 = (tile / tn_count) * BM2, n0 = (tile % tn_count) * BN2;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 2, wn = w & 3;

  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = kend > kbeg ? (kend - kbeg + BK3 - 1) / BK3 : 0;
  auto stage = [&](int kt) {
    bf16_t* ta = smem + (kt & 1) * (TA + TB);
    bf16_t* tb = ta + TA;
    const int k0 = kbeg + kt * BK3;
    if (k0 + BK3 <= kend) {
      dma_tile16(ta, A, lda, k0, m0, M);
      dma_tile16(tb, B, ldb, k0, n0, N);
    } else {
      reg_tile16(ta, A, lda, k0, kend, m0, M);
      reg_tile16(tb, B, ldb, k0, kend, n0, N);
    }
  };
  if (nk > 0) stage(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) stage(kt + 1);
    const bf16_t* a_t = smem + (kt & 1) * (TA + TB);
    const bf16_t* b_t = a_t + TA;
#pragma unroll
    for (int ks = 0; ks < BK3 / 32; ++ks) {
      bf16x8 fa[8], fb[4];
#pragma unroll
      for (int b = 0; b < 4; ++b) fb[b] = frag16(b_t, ks * 32, wn * 64 + b * 16, lane);
#pragma unroll
      for (int a = 0; a < 8; ++a) fa[a] = frag16(a_t, ks * 32, wm * 128 + a * 16, lane);
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = mfma16(fa[a], fb[b], acc[a][b]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  float* out = S == 1 ? C : slab + (int64_t)split * M * N;
  const int64_t ldo = S == 1 ? ldc : N;
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int n = n0 + wn * 64 + b * 16 + (lane & 15);
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 128 + a * 16 + 4 * (lane >> 4) + r;
        if (m < M) {
          float* p = out + (int64_t)m * ldo + n;
          if (S == 1) *p += acc[a][b][r];
          else *p = acc[a][b][r];
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Ring variant: the LDS-DMA kernel above waits vmcnt(0) + barrier every K tile, so each tile's DMA
// must land within ONE tile of MFMAs.  Here the 128 KiB of LDS is a NBUF-deep ring of BK = 32 tiles
// and the DMA runs NBUF-1 tiles ahead behind a COUNTED vmcnt (never 0 in the steady state):
//   vmcnt(P * in_flight_after_kt) | barrier | DMA tile kt+NBUF-1 -> slot (kt-1) % NBUF | 16 MFMAs on slot kt
// One barrier per tile both publishes tile kt (everyone's DMA landed) and retires slot kt-1 (everyone's
// reads of it returned before their MFMAs issued).  P = 4 DMA wave-instructions per tile per wave.
// Used when K is a multiple of 32 within every split (no tail tile).
namespace {
constexpr int BKR = 32;

__device__ __forceinline__ void dma_tile32(uint32_t tile_addr, const bf16_t* base, int64_t ld, int k0, int c0,
                                           int cols) {
  // 32 rows x 512 B = 16 wave-instructions of 1 KiB; wave w issues row pairs w and w + 8
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int pair = w + 8 * it;
    const int row = 2 * pair + (lane >> 5);
    const int p = lane & 31;
    const int c = p ^ ((row & 3) << 2);
    int col = c0 + c * 8;
    col = col < cols ? col : cols - 8;
    glds16(base + (int64_t)(k0 + row) * ld + col, __builtin_amdgcn_readfirstlane(tile_addr + pair * 1024));
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else static_assert(N == 0, "unsupported vmcnt");
}
}  // namespace

template <int NBUF>
__global__ void __launch_bounds__(512, 1) wgrad_ring_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                            float* __restrict__ C, float* __restrict__ slab, int M,
                                                            int N, int K, int64_t lda, int64_t ldb, int64_t ldc, int S,
                                                            int kchunk) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  constexpr int TA = BKR * BM2, TB = BKR * BN2;  // elements per operand tile
  constexpr int SLOT_BYTES = (TA + TB) * 2;
  constexpr int P = 4;                            // DMA wave-instructions per tile per wave
  const int tn_count = (N + BN2 - 1) / BN2;
  const int tiles = ((M + BM2 - 1) / BM2) * tn_count;
  const int id = xcd_remap(blockIdx.x, tiles * S);
  const int split = id / tiles, tile = id % tiles;  // one XCD: same K range, neighbouring tiles (L2 reuse)
  const int m0 = (tile / tn_count) * BM2, n0 = (tile % tn_count) * BN2;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15;
  const int wm = w >> 2, wn = w & 3;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf16_t*)smem);

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};

  const int nk = kend > kbeg ? (kend - kbeg) / BKR : 0;
  auto stage = [&](int kt) {
    const uint32_t base = lds0 + (uint32_t)((kt % NBUF) * SLOT_BYTES);
    const int k0 = kbeg + kt * BKR;
    dma_tile32(base, A, lda, k0, m0, M);
    dma_tile32(base + TA * 2, B, ldb, k0, n0, N);
  };
#pragma unroll
  for (int j = 0; j < NBUF - 1; ++j)
    if (j < nk) stage(j);
  for (int kt = 0; kt < nk; ++kt) {
    // tiles issued after kt that may still be in flight: min(NBUF-2, nk-1-kt)
    const int after = min(NBUF - 2, nk - 1 - kt);
    if (after >= 2) wait_vm<2 * P>();
    else if (after == 1) wait_vm<P>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + NBUF - 1 < nk) stage(kt + NBUF - 1);
    const bf16_t* a_t = smem + (kt % NBUF) * (TA + TB);
    const bf16_t* b_t = a_t + TA;
    bf16x8 fa[2][4], fb[2][2];
#pragma unroll
    for (int ks = 0; ks < BKR / 16; ++ks) {
#pragma unroll
      for (int b = 0; b < 2; ++b) fb[ks][b] = frag2(b_t, ks * 16, wn * 64 + b * 32, g, i16);
#pragma unroll
      for (int a = 0; a < 4; ++a) fa[ks][a] = frag2(a_t, ks * 16, wm * 128 + a * 32, g, i16);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < BKR / 16; ++ks)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma32(fa[ks][a], fb[ks][b], acc[a][b]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);  // k-step 0's reads
#pragma unroll
    for (int q = 0; q < 6; ++q) {                         // k-step 1's reads overlap k-step 0's MFMAs
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 10, 0);
  }
  float* out = S == 1 ? C : slab + (int64_t)split * M * N;
  const int64_t ldo = S == 1 ? ldc : N;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n = n0 + wn * 64 + b * 32 + c32;
      if (n >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 128 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M) {
          float* p = out + (int64_t)m * ldo + n;
          if (S == 1) *p += acc[a][b][r];
          else *p = acc[a][b][r];
        }
      }
    }
}


// ---------------------------------------------------------------------------------------------
// Phase-pipelined variant (the production candidate).  Same 256 x 256 tile / 8 waves / 128 x 64 per
// wave, but each 64-deep K tile is consumed in four PHASES, one per C quadrant (64 x 32) of every
// wave, in the snake order (qm, qn) = (0,0) (0,1) (1,1) (1,0).  Each operand tile is stored as two
// HALF tiles, half h = the rows / columns of quadrant index h for ALL waves ([64 k][128] bf16, 256-B
// rows, chunk ^ ((k & 3) << 2)), so a phase only needs the half tiles of its quadrant:
//   phase p of tile t:  DMA one half tile of tile t+1 (order A0 B0 B1 A1)
//                       s_waitcnt vmcnt(4) + barrier   only if the next phase's fragments need a
//                                                      half tile that just landed (p = 0, 1, 3)
//                       ds_read the fragments of phase p+1     (register double buffer)
//                       8 MFMAs 32x32x16 of phase p
// The DMA of a half tile is waited for ~3 phases after issue and the waits are COUNTED (vmcnt(4) =
// the two youngest half tiles stay in flight) instead of a vmcnt(0) per tile; the LDS-read latency of
// a phase hides behind the previous phase's MFMAs.  B-fragment register slots alternate with the
// tile parity so the tile seam needs no extra buffer; the loop is unrolled by two tiles.
namespace {
constexpr int HALF = 64 * 128;  // elements per half tile

// [64 k][128] half tile, 256-B rows, 16-B chunk XOR (k & 3) << 2
__device__ __forceinline__ int hoff(int k, int col) { return k * 128 + (((col >> 3) ^ ((k & 3) << 2)) << 3) + (col & 7); }

__device__ __forceinline__ bf16x8 hfrag(const bf16_t* half, int kbase, int cbase, int g, int i) {
  const int row = kbase + 8 * (g >> 1) + (i >> 2);
  const int col = cbase + 16 * (g & 1) + 4 * (i & 3);
  const sv4 lo = tr_read(&half[hoff(row, col)]);
  const sv4 hi = tr_read(&half[hoff(row + 4, col)]);
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// DMA plan of one half tile of an MN-major operand ([K][ld] rows): 16 wave-instructions of 4 rows x
// 256 B; wave w issues instructions w and w + 8 (rows 4w.. and 32 + 4w..).  Column slot j of half h
// holds logical column  GROUP * (j / SUB) + h * SUB + j % SUB  (SUB = 64 for A: wave row blocks of 128,
// SUB = 32 for B: wave column blocks of 64) -- the quadrant's columns of every wave, contiguous.
template <int SUB>
struct HalfDma {
  uint32_t voff[2];  // per-lane byte offset for half 0 / half 1 (row 4w + lane/16, swizzled chunk)
  __device__ __forceinline__ void init(int64_t ld, int c0, int cols) {
    const int lane = threadIdx.x & 63;
    const int r = lane >> 4, p = lane & 15;
    const int c = p ^ (r << 2);  // logical chunk carried into physical chunk p of row (4w + r), (row & 3) == r
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = c * 8;
      int col = c0 + 2 * SUB * (j / SUB) + h * SUB + (j % SUB);
      col = col < cols ? col : cols - 8;
      voff[h] = (uint32_t)(((int64_t)r * ld + col) * 2);
    }
  }
  __device__ __forceinline__ void issue(const bf16_t* base, int64_t ld, int k0, int h, uint32_t half_addr) const {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int ins = w + 8 * it;
      glds16s(base + (int64_t)(k0 + 4 * ins) * ld, voff[h], half_addr + (uint32_t)(ins * 1024));
    }
  }
};

template <int N>
__device__ __forceinline__ void vm_wait() {
  if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
}  // namespace

__global__ void __launch_bounds__(512, 2) wgrad_phase_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                             float* __restrict__ C, float* __restrict__ slab, int M,
                                                             int N, int K, int64_t lda, int64_t ldb, int64_t ldc,
                                                             int S, int kchunk) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  // buffer b: A half 0, A half 1, B half 0, B half 1  (4 x 16 KiB)
  const int tn_count = (N + BN2 - 1) / BN2;
  const int tiles = ((M + BM2 - 1) / BM2) * tn_count;
  const int id = xcd_remap(blockIdx.x, tiles * S);
  const int split = id / tiles, tile = id % tiles;
  const int m0 = (tile / tn_count) * BM2, n0 = (tile % tn_count) * BN2;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5, c32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15;
  const int wm = w >> 2, wn = w & 3;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf16_t*)smem);

  HalfDma<64> da;
  HalfDma<32> db;
  da.init(lda, m0, M);
  db.init(ldb, n0, N);
  const int nk = kend > kbeg ? (kend - kbeg) / 64 : 0;

  auto half_ptr = [&](int buf, int which) { return smem + (buf * 4 + which) * HALF; };  // which: 0 A0 1 A1 2 B0 3 B1
  auto half_addr = [&](int buf, int which) { return lds0 + (uint32_t)((buf * 4 + which) * HALF * 2); };
  // DMA order inside a tile: A0, B0, B1, A1
  auto dma = [&](int t, int p) {
    const int k0 = kbeg + t * 64, buf = t & 1;
    if (p == 0) da.issue(A, lda, k0, 0, half_addr(buf, 0));
    else if (p == 1) db.issue(B, ldb, k0, 0, half_addr(buf, 2));
    else if (p == 2) db.issue(B, ldb, k0, 1, half_addr(buf, 3));
    else da.issue(A, lda, k0, 1, half_addr(buf, 1));
  };

  f32x16 acc[2][2][2];  // [qm][a][qn]
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int z = 0; z < 2; ++z) acc[x][y][z] = f32x16{};
  bf16x8 fa[2][2][4];  // [A half][a][ks]
  bf16x8 fb[2][4];     // [slot][ks]

  auto load_a = [&](int buf, int qm) {
    const bf16_t* hp = half_ptr(buf, qm);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) fa[qm][a][ks] = hfrag(hp, ks * 16, wm * 64 + a * 32, g, i16);
  };
  auto load_b = [&](int buf, int qn, int slot) {
    const bf16_t* hp = half_ptr(buf, 2 + qn);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) fb[slot][ks] = hfrag(hp, ks * 16, wn * 32, g, i16);
  };
  auto mfmas = [&](int qm, int qn, int slot) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int a = 0; a < 2; ++a) acc[qm][a][qn] = mfma32(fa[qm][a][ks], fb[slot][ks], acc[qm][a][qn]);
    __builtin_amdgcn_s_setprio(0);
  };

  if (nk > 0) {
    dma(0, 0); dma(0, 1); dma(0, 2); dma(0, 3);
    vm_wait<4>();  // A0, B0 of tile 0
    __builtin_amdgcn_s_barrier();
    load_a(0, 0);
    load_b(0, 0, 0);
  }
  // one tile: TP = tile parity (B slot of half qn is qn ^ TP)
  auto step = [&](int t, auto tp_tag) {
    constexpr int TP = decltype(tp_tag)::value;
    const bool next = t + 1 < nk;
    const int buf = t & 1;
    // phase 0: quadrant (0,0); prefetch B1(t)
    if (next) { dma(t + 1, 0); vm_wait<4>(); } else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    load_b(buf, 1, 1 ^ TP);
    mfmas(0, 0, 0 ^ TP);
    // phase 1: quadrant (0,1); prefetch A1(t)
    if (next) { dma(t + 1, 1); vm_wait<4>(); } else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    load_a(buf, 1);
    mfmas(0, 1, 1 ^ TP);
    // phase 2: quadrant (1,1); nothing new (B0(t) still in its slot)
    if (next) dma(t + 1, 2);
    mfmas(1, 1, 1 ^ TP);
    // phase 3: quadrant (1,0); prefetch A0(t+1), B0(t+1) -> slot 0 ^ (TP ^ 1)
    if (next) {
      dma(t + 1, 3);
      vm_wait<4>();
      __builtin_amdgcn_s_barrier();
      load_a(buf ^ 1, 0);
      load_b(buf ^ 1, 0, 1 ^ TP);
    }
    mfmas(1, 0, 0 ^ TP);
  };
  for (int t = 0; t < nk; t += 2) {
    step(t, std::integral_constant<int, 0>{});
    if (t + 1 < nk) step(t + 1, std::integral_constant<int, 1>{});
  }

  float* out = S == 1 ? C : slab + (int64_t)split * M * N;
  const int64_t ldo = S == 1 ? ldc : N;
#pragma unroll
  for (int qm = 0; qm < 2; ++qm)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int qn = 0; qn < 2; ++qn) {
        const int n = n0 + wn * 64 + qn * 32 + c32;
        if (n >= N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 128 + qm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (m < M) {
            float* p = out + (int64_t)m * ldo + n;
            if (S == 1) *p += acc[qm][a][qn][r];
            else *p = acc[qm][a][qn][r];
          }
        }
      }
}

// C[m][n] += sum_s slab[s][m][n]   (fixed summation order)
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slab, float* __restrict__ C, int M,
                                                          int N, int64_t ldc, int S) {
  const int64_t total4 = (int64_t)M * N / 4;
  const int64_t plane = (int64_t)M * N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total4; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * 4;
    const int m = (int)(e / N), n = (int)(e % N);
    float4 s = *reinterpret_cast<const float4*>(slab + e);
    for (int k = 1; k < S; ++k) {
      const float4 t = *reinterpret_cast<const float4*>(slab + k * plane + e);
      s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    float4* cp = reinterpret_cast<float4*>(C + (int64_t)m * ldc + n);
    float4 c = *cp;
    c.x += s.x; c.y += s.y; c.z += s.z; c.w += s.w;
    *cp = c;
  }
}

static int splits_for(int tiles, int K, int bk, int target) {
  int S = target / tiles;
  if (S < 1) S = 1;
  if (S > 16) S = 16;
  while (S > 1 && K / S < 4 * bk) --S;
  return S;
}

// Variant choice: the 256 x 256 kernel (1 workgroup / CU) when the output has >= 8 such tiles,
// else the 128 x 128 kernel.  Returns splits * 2 + (large ? 1 : 0) so the caller can size the slab.
static int plan(int M, int N, int K, int* S_out) {
  const int t256 = ((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2);
  if (t256 >= 8) {
    *S_out = splits_for(t256, K, BK2, 256);
    return 1;
  }
  const int t128 = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  *S_out = splits_for(t128, K, BK, 512);
  return 0;
}

// Number of K splits for this shape (slab workspace = S * M * N floats when S > 1).
ND_API int nd_wgrad_splits(int M, int N, int K) {
  int S;
  plan(M, N, K, &S);
  return S;
}

// A: dY [K, M] (lda), B: X [K, N] (ldb), C: fp32 [M, N] (ldc).  M, N multiples of 8; any K.
ND_API int nd_wgrad(const void* A, const void* B, float* C, float* slab, int M, int N, int K, int64_t lda, int64_t ldb,
                    int64_t ldc, hipStream_t s) {
  if (M % 8 || N % 8 || lda % 8 || ldb % 8 || (ldc % 4)) return (int)hipErrorInvalidValue;
  int S;
  const int large = plan(M, N, K, &S);
  if (S > 1 && slab == nullptr) return (int)hipErrorInvalidValue;
  // ND_WGRAD_VARIANT (A/B runs): "reg" register-staged 256 kernel, "dma0" LDS-DMA without the
  // sched_group_barrier interleave; default: LDS-DMA with the interleave.
  const char* ev = getenv("ND_WGRAD_VARIANT");
  const int variant = (ev && ev[0] == 'r') ? 1 : (ev && ev[0] == 'p') ? 2 : (ev && ev[0] == 'm') ? 3
                      : (ev && ev[0] == 'n') ? 4 : (ev && ev[0] == 'f') ? 5 : 0;
  const bool sched = !(ev && ev[0] == 'd' && ev[3] == '0');
  const int kchunk_r = ((K + S - 1) / S + BKR - 1) / BKR * BKR;
  if (large && variant == 2 && K % BKR == 0) {
    const int tiles = ((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2);
    constexpr int NB = 4;
    const size_t lds = (size_t)NB * BKR * (BM2 + BN2) * sizeof(bf16_t);  // 128 KiB
    static const hipError_t attr_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_ring_kernel<NB>),
                                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)attr_ok;
    hipLaunchKernelGGL(wgrad_ring_kernel<NB>, dim3(tiles * S), dim3(512), lds, s, (const bf16_t*)A, (const bf16_t*)B,
                       C, slab, M, N, K, lda, ldb, ldc, S, kchunk_r);
  } else if (large && variant == 5 && K % 64 == 0) {  // "fph": phase-pipelined
    const int kchunk = ((K + S - 1) / S + 63) / 64 * 64;
    const int tiles = ((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2);
    const size_t lds = 8 * (size_t)HALF * sizeof(bf16_t);  // 128 KiB
    static const hipError_t attr_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_phase_kernel),
                                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)attr_ok;
    hipLaunchKernelGGL(wgrad_phase_kernel, dim3(tiles * S), dim3(512), lds, s, (const bf16_t*)A, (const bf16_t*)B, C,
                       slab, M, N, K, lda, ldb, ldc, S, kchunk);
  } else if (large && variant == 4) {  // "nodma": compute-only diagnostic
    const int kchunk = ((K + S - 1) / S + BK3 - 1) / BK3 * BK3;
    const int tiles = ((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2);
    const size_t lds = 2 * (size_t)BK3 * (BM2 + BN2) * sizeof(bf16_t);
    static const hipError_t attr_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_dma_kernel<true, true>),
                                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)attr_ok;
    hipLaunchKernelGGL((wgrad_dma_kernel<true, true>), dim3(tiles * S), dim3(512), lds, s, (const bf16_t*)A,
                       (const bf16_t*)B, C, slab, M, N, K, lda, ldb, ldc, S, kchunk);
  } else if (large && variant == 3) {
    const int kchunk = ((K + S - 1) / S + BK3 - 1) / BK3 * BK3;
    const int tiles = ((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2);
    const size_t lds = 2 * (size_t)BK3 * (BM2 + BN2) * sizeof(bf16_t);  // 128 KiB
    static const hipError_t attr_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_m16_kernel),
                                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)attr_ok;
    hipLaunchKernelGGL(wgrad_m16_kernel, dim3(tiles * S), dim3(512), lds, s, (const bf16_t*)A, (const bf16_t*)B, C,
                       slab, M, N, K, lda, ldb, ldc, S, kchunk);
  } else if (large && variant != 1 && M >= 8 && N >= 8) {
    const int kchunk = ((K + S - 1) / S + BK3 - 1) / BK3 * BK3;
    const int tiles = ((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2);
    const size_t lds = 2 * (size_t)BK3 * (BM2 + BN2) * sizeof(bf16_t);  // 128 KiB
    static const hipError_t attr_ok =
        (hipError_t)(hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_dma_kernel<true>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) |
                     hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_dma_kernel<false>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    (void)attr_ok;
    if (sched)
      hipLaunchKernelGGL(wgrad_dma_kernel<true>, dim3(tiles * S), dim3(512), lds, s, (const bf16_t*)A,
                         (const bf16_t*)B, C, slab, M, N, K, lda, ldb, ldc, S, kchunk);
    else
      hipLaunchKernelGGL(wgrad_dma_kernel<false>, dim3(tiles * S), dim3(512), lds, s, (const bf16_t*)A,
                         (const bf16_t*)B, C, slab, M, N, K, lda, ldb, ldc, S, kchunk);
  } else if (large) {
    const int kchunk = ((K + S - 1) / S + BK2 - 1) / BK2 * BK2;
    const int tiles = ((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2);
    const size_t lds = 2 * (size_t)BK2 * (BM2 + BN2) * sizeof(bf16_t);
    hipLaunchKernelGGL(wgrad256_kernel, dim3(tiles * S), dim3(512), lds, s, (const bf16_t*)A, (const bf16_t*)B, C,
                       slab, M, N, K, lda, ldb, ldc, S, kchunk);
  } else {
    const int kchunk = ((K + S - 1) / S + BK - 1) / BK * BK;
    const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    hipLaunchKernelGGL(wgrad_kernel, dim3(tiles * S), dim3(256), 0, s, (const bf16_t*)A, (const bf16_t*)B, C, slab, M,
                       N, K, lda, ldb, ldc, S, kchunk);
  }
  if (S > 1) {
    int64_t blocks = ((int64_t)M * N / 4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, slab, C, M, N, ldc, S);
  }
  ND_LAUNCH_CHECK();
}
