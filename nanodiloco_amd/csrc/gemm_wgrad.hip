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
//   * XCD-aware block remap so the workgroups sharing an A row-panel run on one XCD's L2.
//
// Kernels in this file (dispatch: nd_wgrad / nd_wgrad2 / nd_wgrad_f8 at the end):
//   wgrad_pp_kernel    the default (K % 64 == 0, >= 8 output tiles of 256 x 256): ping-pong pairing of
//                      csrc/gemm_pp.hip, LDS-DMA staging, counted vmcnt; one or TWO products per launch
//                      (nd_wgrad2, round 5: e.g. the MLP's down + gate|up gradients fill the chip together)
//   wgrad_dma_kernel   256 x 256, 4-wave-pair LDS-DMA kernel of round 2: K % 64 != 0 (register-staged tail)
//                      and the dma0 / dmas A/B variants
//   wgrad_kernel       128 x 128 per 256-thread workgroup (2 x 2 waves of 64 x 64, 32x32x16 MFMA),
//                      register-staged prefetch: outputs with < 8 tiles of 256 x 256
//   wgrad8_pp_kernel   the fp8 form of the ping-pong kernel (e5m2 / e4m3 dY, e4m3 X, 16x16x128 f8f6f4 MFMA)
// Split count per launch: a fixed rule (~256 workgroups), replaced by a makespan model where it predicts a
// >= 10 % win (plan() below).
#include "common.h"
#include <cstdlib>
#include <cstring>


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
// 256 x 256 tile geometry and the transposing fragment helpers of the LDS-DMA kernel below (8 waves as
// 2 (M) x 4 (N), 128 x 64 each).  (The round-2 register-staged 256 x 256 kernel and the round-3 4-wave
// AGPR variant that used to sit here measured slower than the ping-pong kernel; removed in round 5.)
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
}  // namespace

// ---------------------------------------------------------------------------------------------
// LDS-DMA kernel (round 2; since round 3 the path for K % 64 != 0 and the dma0 / dmas A/B variants): same
// 256 x 256 / 8-wave / 128 x 64-per-wave geometry, but tiles move global -> LDS with global_load_lds_dwordx4 (no VGPR round trip, no ds_write issue cost,
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

// =====================================================================================================
// Ping-pong weight-gradient kernel (round 3, the default for K % 64 == 0): the pairing of
// csrc/gemm_pp.hip applied to C (+)= A^T B.  8 waves, 256 x 256 tile; group g = w / 4 owns output rows
// m 128 g .. + 127, wave w % 4 the 64 columns n 64 (w % 4) .. + 63 (8 x 4 v_mfma_f32_16x16x32_bf16
// accumulators, 128 VGPRs, + one K-tile of fragments, 96 VGPRs: 2 waves / SIMD).  Each 64-token K-tile
// is a LOAD phase (all 48 transposing fragment reads of the K-tile + this group's LDS-DMA pieces) and a
// COMPUTE phase (64 MFMAs), group 1 one barrier behind group 0, so the two waves of a SIMD alternate
// matrix work and loads.  The LDS image holds the operands as they lie in memory ([k][m] / [k][n]
// half-tiles of 64 rows x 256 B, 16-B chunk index ^ f(row), f = ((row & 3) << 2) ^ (((row >> 3) & 1) << 1):
// the 32 lanes of one ds_read_b64_tr_b16 read rows q and q + 8 (q = 0..3) at one 32-B column pair
// -> 8 distinct 32-B bank segments).  DMA ownership and counted waits are those of gemm_pp_kernel:
// group 0 stages B (both halves) of K-tile s + 1 in LOAD(s) and retires it at the end of COMPUTE(s);
// group 1 stages A1 of s + 1 and A0 of s + 2, retiring A0(s + 1) at the end of LOAD(s) and A1(s + 1)
// at the end of COMPUTE(s).  One (tile, K-split) per workgroup; split-K slabs as wgrad_dma_kernel.
namespace {
constexpr uint32_t WPP_HALF_B = 64 * 128 * 2;  // [64 k][128 cols] bf16
constexpr uint32_t WPP_BUF_B = 4 * WPP_HALF_B;  // A0 A1 B0 B1 = 64 KiB

__device__ __forceinline__ uint32_t wpp_off(int row, int ch) {
  return (uint32_t)(row * 256 + ((ch ^ (((row & 3) << 2) ^ (((row >> 3) & 1) << 1))) << 4));
}
// 16x16x32 operand, the column (m or n) on the lane: lane l -> column c0 + (l & 15), k = kb + 8 (l >> 4) + j
__device__ __forceinline__ bf16x8 wpp_frag(const char* half, int kb, int c0, int lane) {
  const int gg = lane >> 4, i = lane & 15;
  const int row = kb + 8 * gg + (i >> 2), col = c0 + 4 * (i & 3);
  const char* p = half + wpp_off(row, col >> 3) + (col & 7) * 2;
  const sv4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((sv4 __attribute__((address_space(3)))*)(p));
  const sv4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((sv4 __attribute__((address_space(3)))*)(p + 1024));
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}
__device__ __forceinline__ f32x4 wpp_mma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0, 0);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wpp_rsrc(const void* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0,
                                           (int)(bytes > 0 ? (bytes < 0x7ffffffe ? bytes : 0x7ffffffe) : 0), 0x00020000);
}
__device__ __forceinline__ void wpp_dma(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(r), "s"(lds) : "memory");
}
// FLAT-global form (SGPR base + 32-bit per-lane offset, no range check): half-tiles whose 128 columns exist
__device__ __forceinline__ void wpp_gdma(const void* base, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(base), "s"(lds) : "memory");
}
__device__ __forceinline__ void wpp_bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}
template <int N> __device__ __forceinline__ void wpp_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }
__device__ __forceinline__ void wpp_vmn(int n) {  // n in {0, 4, 8}
  if (n >= 8) wpp_vm<8>();
  else if (n >= 4) wpp_vm<4>();
  else wpp_vm<0>();
}
}  // namespace

// One weight-gradient product of a (possibly grouped) launch: C[M, N] (+)= A^T B, A [K, M], B [K, N].
struct WgProb {
  const bf16_t* A;
  const bf16_t* B;
  float* C;
  float* slab;
  int M, N;
  int64_t lda, ldb, ldc;
};

// ABL (timing ablations, wrong results; ND_WGRAD_VARIANT=a<bits>): 1 no LDS-DMA in the loop, 2 fragments read
// only for the first K-tile, 4 no barriers in the loop, 8 no vmcnt waits in the loop, 16 no MFMAs
//
// Grouped launch (round 5): workgroups [0, nwg0) run product p0, the rest p1 (same K and split count S).
// Two products whose tile counts alone leave CUs idle fill the chip together: the Llama-150M MLP's
// down (44 tiles) and gate|up (84) weight gradients are 220 + 252 workgroups as separate launches
// (S = 5 / 3) but exactly 256 as one launch with S = 2.
template <bool GD, int ABL = 0>
__global__ void __launch_bounds__(512, 1) wgrad_pp_kernel(WgProb p0, WgProb p1, int nwg0, int K, int S, int kchunk) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem_bf[];
  char* smem = reinterpret_cast<char*>(smem_bf);
  const int gid = xcd_remap(blockIdx.x, gridDim.x);
  const bool second = gid >= nwg0;
  const bf16_t* __restrict__ A = second ? p1.A : p0.A;
  const bf16_t* __restrict__ B = second ? p1.B : p0.B;
  float* __restrict__ C = second ? p1.C : p0.C;
  float* __restrict__ slab = second ? p1.slab : p0.slab;
  const int M = second ? p1.M : p0.M, N = second ? p1.N : p0.N;
  const int64_t lda = second ? p1.lda : p0.lda, ldb = second ? p1.ldb : p0.ldb, ldc = second ? p1.ldc : p0.ldc;
  const int tn_count = (N + 255) / 256;
  const int tiles = ((M + 255) / 256) * tn_count;
  const int id = second ? gid - nwg0 : gid;
  const int split = id / tiles, tile = id % tiles;
  const int m0 = (tile / tn_count) * 256, n0 = (tile % tn_count) * 256;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nk = (kend - kbeg) / 64;  // host: K % 64 == 0, kchunk % 64 == 0, every split non-empty
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = w >> 2, wn = w & 3;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);

  // DMA: piece q of this wave = half-tile rows 4 j .. 4 j + 3 (j = wn + 4 q); lane -> row 4 j + lane / 16,
  // physical chunk lane & 15 <- logical chunk (lane & 15) ^ f(row), f independent of q
  const int64_t ld = g == 0 ? ldb : lda;
  const int fsw = ((lane >> 4) << 2) ^ (((wn >> 1) & 1) << 1);
  uint32_t voff[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = 4 * (wn + 4 * q) + (lane >> 4);
    voff[q] = (uint32_t)(((int64_t)row * ld + (((lane & 15) ^ fsw) << 3)) * 2);
  }
  // half h of operand (g == 0: B columns n0 + 128 h .., g == 1: A columns m0 + 128 h ..) of K-tile kt
  auto stage = [&](int kt, int h) __attribute__((always_inline)) {
    const int64_t e0 = (int64_t)(kbeg + 64 * kt) * ld + (g == 0 ? n0 : m0) + 128 * h;
    const uint32_t dst = lds0 + (uint32_t)(kt & 1) * WPP_BUF_B + (uint32_t)(g == 0 ? 2 + h : h) * WPP_HALF_B +
                         (uint32_t)wn * 1024u;
    if (GD && (g == 0 ? n0 + 128 * h + 128 <= N : m0 + 128 * h + 128 <= M)) {
      if constexpr (ND_DMA_BURST) {
        gdma4<4096>((g == 0 ? B : A) + e0, voff[0], voff[1], voff[2], voff[3], dst);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) wpp_gdma((g == 0 ? B : A) + e0, voff[q], dst + (uint32_t)q * 4096u);
      }
    } else {
      const auto r = wpp_rsrc((g == 0 ? B : A) + e0, ((int64_t)K * ld - e0) * 2);
      if constexpr (ND_DMA_BURST) {
        dma4<4096>(r, voff[0], voff[1], voff[2], voff[3], dst);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) wpp_dma(r, voff[q], dst + (uint32_t)q * 4096u);
      }
    }
  };
  bf16x8 fa[8][2], fb[4][2];
  auto load_frags = [&](int kt) __attribute__((always_inline)) {
    const char* base = smem + (kt & 1) * WPP_BUF_B;
    const char* ah = base + g * WPP_HALF_B;
    const char* bh = base + (2 + (wn >> 1)) * WPP_HALF_B;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int b = 0; b < 4; ++b) fb[b][ks] = wpp_frag(bh, 32 * ks, (wn & 1) * 64 + 16 * b, lane);
#pragma unroll
      for (int a = 0; a < 8; ++a) fa[a][ks] = wpp_frag(ah, 32 * ks, 16 * a, lane);
    }
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: K-tile 0 and A0 of K-tile 1, drained; group 1 one barrier behind
  if (g == 0) {
    stage(0, 0);
    stage(0, 1);
  } else {
    stage(0, 0);
    stage(0, 1);
    if (nk > 1) stage(1, 0);
  }
  wpp_vm<0>();
  wpp_bar();
  if (g == 1) wpp_bar();
  for (int s = 0; s < nk; ++s) {
    const bool more1 = s + 1 < nk, more2 = s + 2 < nk;
    // ================= LOAD(s)
    if (ABL & 1) {
    } else if (g == 0) {
      if (more1) {
        stage(s + 1, 0);
        stage(s + 1, 1);
      }
    } else {
      if (more1) stage(s + 1, 1);  // A1(s + 1)
      if (more2) stage(s + 2, 0);  // A0(s + 2)
    }
    if (!(ABL & 2) || s == 0) load_frags(s);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (g == 1 && !(ABL & 8)) wpp_vmn((more1 ? 4 : 0) + (more2 ? 4 : 0));  // A0(s + 1) landed
    if (!(ABL & 4)) wpp_bar();
    // ================= COMPUTE(s)
    __builtin_amdgcn_s_setprio(1);
    if constexpr ((ABL & 16) != 0) {
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) asm volatile("" ::"v"(fa[a][0]), "v"(fb[b][1]));
    } else {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = wpp_mma(fa[a][ks], fb[b][ks], acc[a][b]);
    }
    __builtin_amdgcn_s_setprio(0);
    if (ABL & 8) {
    } else if (g == 0) wpp_vm<0>();     // B(s + 1) landed
    else wpp_vmn(more2 ? 4 : 0);        // A1(s + 1) landed
    if (!(ABL & 4)) wpp_bar();
  }
  if (ABL & 9) wpp_vm<0>();
  // epilogue: acc[a][b] lane l reg r = C[m0 + 128 g + 16 a + 4 (l >> 4) + r][n0 + 64 wn + 16 b + (l & 15)].
  // Both groups first meet at the same barrier (group 1 ran one more), after which every LDS read and
  // LDS-DMA write of the K-loop is done; each wave then transposes its 128 x 64 block through a private
  // 16-KiB LDS region (two 64-row halves, 16-B chunk ^ (row & 15)) so the slab / C rows go out as
  // 16-B-per-lane, 256-B-per-row stores instead of 4-B scalar ones.
  if (g == 0) wpp_bar();  // group 1 ran one barrier more
  float* out = S == 1 ? C : slab + (int64_t)split * M * N;
  const int64_t ldo = S == 1 ? ldc : N;
  float* reg = reinterpret_cast<float*>(smem) + w * (64 * 64);
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * a + 4 * (lane >> 4) + r, col = 16 * b + (lane & 15);
          reg[row * 64 + (((col >> 2) ^ (row & 15)) << 2) + (col & 3)] = acc[4 * half + a][b][r];
        }
    asm volatile("" ::: "memory");
    const int c4 = lane & 15;
    const int n = n0 + wn * 64 + 4 * c4;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = 4 * i + (lane >> 4);
      const float4 v = *reinterpret_cast<const float4*>(reg + row * 64 + ((c4 ^ (row & 15)) << 2));
      const int m = m0 + g * 128 + 64 * half + row;
      if (m < M && n < N) {
        float4* p = reinterpret_cast<float4*>(out + (int64_t)m * ldo + n);
        if (S == 1) {
          float4 c = *p;
          c.x += v.x; c.y += v.y; c.z += v.z; c.w += v.w;
          *p = c;
        } else {
          *p = v;
        }
      }
    }
    asm volatile("" ::: "memory");
  }
}

// =====================================================================================================
// fp8 weight-gradient kernel (round 4): C (+)= sa sb dY8^T X8 with dY8 [K, M] (e5m2 or e4m3) and X8 [K, N]
// (e4m3) as the producers wrote them (token-major, no transposed copies).  wgrad_pp_kernel's ping-pong
// structure with the K-tile doubled to 128 tokens, so the LDS image (128 k-rows x 128 B per half-tile), the
// DMA pieces (8 rows x 128 B) and the per-K-tile instruction counts stay those of the bf16 kernel while
// each K-tile carries twice the work: 48 ds_read_b64_tr_b8 per wave (4 per fragment: 8 k-rows of 16
// columns each, the lane's 32 K bytes) and 32 v_mfma_scale_f32_16x16x128_f8f6f4 (twice the bf16 rate).
// LDS chunk swizzle f(r) = ((r >> 1) & 3) ^ (((r >> 5) & 1) << 2): the two 16-lane groups of a 32-lane half
// read rows 32 apart, 8 rows x 16 B each -> 16 distinct 4-bank sets (conflict-free).
namespace {
constexpr uint32_t W8_HALF_B = 128 * 128;      // [128 k][128 cols] bytes
constexpr uint32_t W8_BUF_B = 4 * W8_HALF_B;   // A0 A1 B0 B1 = 64 KiB
typedef int w8v2 __attribute__((ext_vector_type(2)));
typedef int w8v8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int w8_swz(int r) { return ((r >> 1) & 3) ^ (((r >> 5) & 1) << 2); }
// 16x16x128 operand, the column on the lane: lane l -> column c0 + (l & 15), k = 32 (l >> 4) + 0 .. 31
__device__ __forceinline__ w8v8 w8_frag(const char* half, int c0, int lane) {
  const int gq = lane >> 4, j = lane & 15, q = j >> 1, p = j & 1;
  const int ch = c0 >> 4;  // c0 % 16 == 0
  w8v8 r;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int row = 32 * gq + 8 * t + q;
    const char* a = half + row * 128 + ((ch ^ w8_swz(row)) << 4) + 8 * p;
    const w8v2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((w8v2 __attribute__((address_space(3)))*)(a));
    r[2 * t] = v[0];
    r[2 * t + 1] = v[1];
  }
  return r;
}
}  // namespace

// FA: dY's format (0 e4m3, 1 e5m2); X is e4m3
template <int FA>
__global__ void __launch_bounds__(512, 1) wgrad8_pp_kernel(const uint8_t* __restrict__ A, const uint8_t* __restrict__ B,
                                                           float* __restrict__ C, float* __restrict__ slab, int M, int N,
                                                           int K, int64_t lda, int64_t ldb, int64_t ldc, int S,
                                                           int kchunk, const float* __restrict__ sa,
                                                           const float* __restrict__ sb) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem_bf[];
  char* smem = reinterpret_cast<char*>(smem_bf);
  const int tn_count = (N + 255) / 256;
  const int tiles = ((M + 255) / 256) * tn_count;
  const int id = xcd_remap(blockIdx.x, tiles * S);
  const int split = id / tiles, tile = id % tiles;
  const int m0 = (tile / tn_count) * 256, n0 = (tile % tn_count) * 256;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nk = (kend - kbeg) / 128;  // host: K % 128 == 0, kchunk % 128 == 0, every split non-empty
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = w >> 2, wn = w & 3;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem);
  const float sc = sa[0] * sb[0];

  // DMA piece q of this wave = half-tile k-rows 8 j .. 8 j + 7 (j = wn + 4 q); lane -> row 8 j + lane / 8,
  // physical chunk lane & 7 <- logical chunk (lane & 7) ^ f(row)
  const int64_t ld = g == 0 ? ldb : lda;
  uint32_t voff[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = 8 * (wn + 4 * q) + (lane >> 3);
    voff[q] = (uint32_t)((int64_t)row * ld + (((lane & 7) ^ w8_swz(row)) << 4));
  }
  auto stage = [&](int kt, int h) __attribute__((always_inline)) {
    const int64_t e0 = (int64_t)(kbeg + 128 * kt) * ld + (g == 0 ? n0 : m0) + 128 * h;
    const uint32_t dst = lds0 + (uint32_t)(kt & 1) * W8_BUF_B + (uint32_t)(g == 0 ? 2 + h : h) * W8_HALF_B +
                         (uint32_t)wn * 1024u;
    if (g == 0 ? n0 + 128 * h + 128 <= N : m0 + 128 * h + 128 <= M) {
#pragma unroll
      for (int q = 0; q < 4; ++q) wpp_gdma((g == 0 ? B : A) + e0, voff[q], dst + (uint32_t)q * 4096u);
    } else {
      const auto r = wpp_rsrc((g == 0 ? B : A) + e0, (int64_t)K * ld - e0);
#pragma unroll
      for (int q = 0; q < 4; ++q) wpp_dma(r, voff[q], dst + (uint32_t)q * 4096u);
    }
  };
  w8v8 fa[8], fb[4];
  auto load_frags = [&](int kt) __attribute__((always_inline)) {
    const char* base = smem + (kt & 1) * W8_BUF_B;
    const char* ah = base + g * W8_HALF_B;
    const char* bh = base + (2 + (wn >> 1)) * W8_HALF_B;
#pragma unroll
    for (int b = 0; b < 4; ++b) fb[b] = w8_frag(bh, (wn & 1) * 64 + 16 * b, lane);
#pragma unroll
    for (int a = 0; a < 8; ++a) fa[a] = w8_frag(ah, 16 * a, lane);
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (g == 0) {
    stage(0, 0);
    stage(0, 1);
  } else {
    stage(0, 0);
    stage(0, 1);
    if (nk > 1) stage(1, 0);
  }
  wpp_vm<0>();
  wpp_bar();
  if (g == 1) wpp_bar();
  for (int s = 0; s < nk; ++s) {
    const bool more1 = s + 1 < nk, more2 = s + 2 < nk;
    // ================= LOAD(s)
    if (g == 0) {
      if (more1) {
        stage(s + 1, 0);
        stage(s + 1, 1);
      }
    } else {
      if (more1) stage(s + 1, 1);  // A1(s + 1)
      if (more2) stage(s + 2, 0);  // A0(s + 2)
    }
    load_frags(s);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (g == 1) wpp_vmn((more1 ? 4 : 0) + (more2 ? 4 : 0));  // A0(s + 1) landed
    wpp_bar();
    // ================= COMPUTE(s)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa[a], fb[b], acc[a][b], FA, 0, 0, 0x7f7f7f7f, 0,
                                                                     0x7f7f7f7f);
    __builtin_amdgcn_s_setprio(0);
    if (g == 0) wpp_vm<0>();            // B(s + 1) landed
    else wpp_vmn(more2 ? 4 : 0);        // A1(s + 1) landed
    wpp_bar();
  }
  // epilogue: wgrad_pp_kernel's (acc[a][b] lane l reg r = C[m0 + 128 g + 16 a + 4 (l >> 4) + r]
  // [n0 + 64 wn + 16 b + (l & 15)]), dequantised by sc
  if (g == 0) wpp_bar();
  float* out = S == 1 ? C : slab + (int64_t)split * M * N;
  const int64_t ldo = S == 1 ? ldc : N;
  float* reg = reinterpret_cast<float*>(smem) + w * (64 * 64);
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * a + 4 * (lane >> 4) + r, col = 16 * b + (lane & 15);
          reg[row * 64 + (((col >> 2) ^ (row & 15)) << 2) + (col & 3)] = acc[4 * half + a][b][r] * sc;
        }
    asm volatile("" ::: "memory");
    const int c4 = lane & 15;
    const int n = n0 + wn * 64 + 4 * c4;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = 4 * i + (lane >> 4);
      const float4 v = *reinterpret_cast<const float4*>(reg + row * 64 + ((c4 ^ (row & 15)) << 2));
      const int m = m0 + g * 128 + 64 * half + row;
      if (m < M && n < N) {
        float4* p = reinterpret_cast<float4*>(out + (int64_t)m * ldo + n);
        if (S == 1) {
          float4 c = *p;
          c.x += v.x; c.y += v.y; c.z += v.z; c.w += v.w;
          *p = c;
        } else {
          *p = v;
        }
      }
    }
    asm volatile("" ::: "memory");
  }
}

// ND_WGRAD_PLAN=old: the fixed split rule only; =c<pct>: take the makespan model's split count when it predicts
// a time below pct % of the fixed rule's (default 90; A/B of the threshold).  The model is only trusted for large
// predicted gains: at 99 % it moves the Llama-150M q|k|v weight gradient from 5 to 16 splits (3 full waves) and
// the bf16 step gets 2.1 % SLOWER (session r5al)
static const double g_wgrad_plan_thr = [] {
  const char* e = getenv("ND_WGRAD_PLAN");
  if (e && e[0] == 'o') return 0.0;
  if (e && e[0] == 'c' && atoi(e + 1) > 0) return atoi(e + 1) / 100.0;
  return 0.9;
}();

static int num_cus_wg() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      return 256;
    return v;
  }();
  return n;
}

static bool wgrad_pp_eligible(int M, int N, int K, int64_t lda, int64_t ldb, int64_t ldc) {
  return M % 8 == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0 && K % 64 == 0 && K > 0 &&
         ((M + 255) / 256) * ((N + 255) / 256) >= 8 && (int64_t)64 * (lda > ldb ? lda : ldb) * 2 < (1ll << 31);
}

static double split_cost(int T, int K, int64_t mn_total, int S) {
  const int nk = K / 64, ncu = num_cus_wg();
  const double waves = (double)((T * S + ncu - 1) / ncu);
  return waves * (double)((nk + S - 1) / S) + (S > 1 ? (double)(S + 2) * mn_total * 4.0 / 8.95e6 : 0.0);
}

static int group_splits(int T, int K, int64_t mn_total) {
  const int nk = K / 64;
  int best = 1;
  double best_cost = 1e300;
  for (int S = 1; S <= 16; ++S) {
    if (S > 1 && nk / S < 4) break;
    const double cost = split_cost(T, K, mn_total, S);
    if (cost < best_cost * 0.999) {
      best_cost = cost;
      best = S;
    }
  }
  return best;
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
// A/B hook (scripts/wgrad_splits_ab.py): force the split count of single weight gradients (0 = the plan)
static int g_wgrad_force_s = 0;
ND_API int nd_wgrad_force_splits(int s) {
  const int old = g_wgrad_force_s;
  g_wgrad_force_s = s > 0 ? (s > 16 ? 16 : s) : 0;
  return old;
}

static int plan(int M, int N, int K, int* S_out, bool use_cost = true) {
  const int t256 = ((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2);
  if (t256 >= 8) {
    int S = splits_for(t256, K, BK2, 256);
    // the makespan model of the grouped launch, taken only when it predicts >= 10 % (idle CUs clock the
    // busy ones up, so small predicted gains do not materialise: profiles/r5_gemm_tokens.md); e.g. the
    // Llama-1B down-projection gradient: 176 tiles -> S = 4 instead of 176 workgroups on 256 CUs (bf16
    // step +1.7 %).  Not for the fp8 kernel (use_cost = false): its side-stream wgrads share the chip with
    // unfenced own GEMMs, and the 1B fp8 step measured 0.973x with the model
    if (use_cost && g_wgrad_plan_thr > 0.0 && K % 64 == 0) {
      const int Sc = group_splits(t256, K, (int64_t)M * N);
      if (split_cost(t256, K, (int64_t)M * N, Sc) < g_wgrad_plan_thr * split_cost(t256, K, (int64_t)M * N, S)) S = Sc;
    }
    if (g_wgrad_force_s > 0) S = g_wgrad_force_s;
    *S_out = S;
    return 1;
  }
  const int t128 = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  *S_out = splits_for(t128, K, BK, 512);
  return 0;
}

// K range per split, rounded up to whole bk tiles; S shrinks until every split owns at least one
// tile (with the rounding, the last split could otherwise be empty -- e.g. K = 41 * 64, S = 8 -- and
// its slab plane would never be written while slab_reduce_kernel still sums all S planes)
static int fit_kchunk(int K, int* S, int bk) {
  for (;;) {
    const int kchunk = ((K + *S - 1) / *S + bk - 1) / bk * bk;
    if (*S <= 1 || (int64_t)(*S - 1) * kchunk < K) return kchunk;
    --*S;
  }
}

// ND_WGRAD_VARIANT (A/B runs), read once at load; outside -DND_ABLATION builds the wrong-result forms
// ("nodma", "a<bits>") are dropped, i.e. the default kernel runs
static const char* wgrad_env() {
  static const char* v = [] {
    const char* e = getenv("ND_WGRAD_VARIANT");
#ifndef ND_ABLATION
    if (e && (e[0] == 'n' || e[0] == 'a')) return (const char*)nullptr;
#endif
    return e;
  }();
  return v;
}

// Number of K splits for this shape (slab workspace = S * M * N floats when S > 1).
ND_API int nd_wgrad_splits(int M, int N, int K) {
  int S;
  plan(M, N, K, &S);
  return S;
}

// The same for the fp8 weight-gradient kernel (nd_wgrad_f8).
ND_API int nd_wgrad_f8_splits(int M, int N, int K) {
  int S;
  plan(M, N, K, &S, false);
  return S;
}

// A: dY [K, M] (lda), B: X [K, N] (ldb), C: fp32 [M, N] (ldc).  M, N multiples of 8; any K.
ND_API int nd_wgrad(const void* A, const void* B, float* C, float* slab, int M, int N, int K, int64_t lda, int64_t ldb,
                    int64_t ldc, hipStream_t s) {
  if (M % 8 || N % 8 || lda % 8 || ldb % 8 || (ldc % 4)) return (int)hipErrorInvalidValue;
  int S;
  const int large = plan(M, N, K, &S);
  if (S > 1 && slab == nullptr) return (int)hipErrorInvalidValue;
  // ND_WGRAD_VARIANT (A/B runs, read once when the library loads): "dma0" the round-2 LDS-DMA kernel,
  // compiler-scheduled; "dmas" the same with the sched_group_barrier interleave (MFMA / 2 transposing reads:
  // measured 4-13 % SLOWER per kernel, -1.7 % e2e); "b" the ping-pong kernel with buffer-form pieces only;
  // "nodma" / "a<bits>" timing ablations with wrong results (-DND_ABLATION builds only).  (Measured and
  // dropped, see docs/DESIGN.md: s_setprio around the MFMA clusters, a 4-deep BK=32 ring with counted vmcnt,
  // a 16x16x32-MFMA version, a quadrant-phase pipeline, the register-staged 256 x 256 kernel and the 4-wave
  // AGPR kernel -- the last two removed in round 5.)
  const char* ev = wgrad_env();
  const bool sched = ev && strncmp(ev, "dmas", 4) == 0;
  const bool pp = large && M >= 8 && N >= 8 && K % 64 == 0 && (int64_t)64 * (lda > ldb ? lda : ldb) * 2 < (1ll << 31) &&
                 !(ev && (ev[0] == 'd' || ev[0] == 'n'));
  if (pp) {  // default: ping-pong kernel (ND_WGRAD_VARIANT=dma0 / dmas select the LDS-DMA kernel)
    const int kchunk = fit_kchunk(K, &S, 64);
    const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
    const size_t lds = 2 * (size_t)WPP_BUF_B;  // 128 KiB
    static const hipError_t attrp =
        (hipError_t)(hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_pp_kernel<false>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) |
                     hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_pp_kernel<true>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if (attrp != hipSuccess) return (int)attrp;
    const WgProb prob{(const bf16_t*)A, (const bf16_t*)B, C, slab, M, N, lda, ldb, ldc};
#ifdef ND_ABLATION
    if (ev && ev[0] == 'a') {  // timing ablations (wrong results)
      const int abl = atoi(ev + 1);
#define ND_WA(X) case X: hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_pp_kernel<true, X>), \
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
  hipLaunchKernelGGL((wgrad_pp_kernel<true, X>), dim3(tiles * S), dim3(512), lds, s, prob, prob, tiles * S, K, S, \
                     kchunk); break;
      switch (abl) { ND_WA(1) ND_WA(2) ND_WA(4) ND_WA(8) ND_WA(16) ND_WA(3) ND_WA(7) ND_WA(15) ND_WA(31) default: return (int)hipErrorInvalidValue; }
#undef ND_WA
      ND_LAUNCH_CHECK();
    }
#endif
    // default: full half-tiles staged with FLAT-global LDS loads (bitwise the same as the buffer form,
    // 1.005x over the three Llama-150M shapes, profiles/r4_gdma_ab.md); "b": buffer loads only (A/B)
    if (!(ev && ev[0] == 'b'))
      hipLaunchKernelGGL(wgrad_pp_kernel<true>, dim3(tiles * S), dim3(512), lds, s, prob, prob, tiles * S, K, S, kchunk);
    else
      hipLaunchKernelGGL(wgrad_pp_kernel<false>, dim3(tiles * S), dim3(512), lds, s, prob, prob, tiles * S, K, S, kchunk);
#ifdef ND_ABLATION
  } else if (large && ev && ev[0] == 'n') {  // "nodma": compute-only diagnostic (wrong result)
    const int kchunk = fit_kchunk(K, &S, BK3);
    const int tiles = ((M + BM2 - 1) / BM2) * ((N + BN2 - 1) / BN2);
    const size_t lds = 2 * (size_t)BK3 * (BM2 + BN2) * sizeof(bf16_t);
    static const hipError_t attr_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_dma_kernel<true, true>),
                                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    (void)attr_ok;
    hipLaunchKernelGGL((wgrad_dma_kernel<true, true>), dim3(tiles * S), dim3(512), lds, s, (const bf16_t*)A,
                       (const bf16_t*)B, C, slab, M, N, K, lda, ldb, ldc, S, kchunk);
#endif
  } else if (large) {  // K % 64 != 0 (register-staged K tail) or ND_WGRAD_VARIANT=dma0 / dmas
    const int kchunk = fit_kchunk(K, &S, BK3);
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
  } else {
    const int kchunk = fit_kchunk(K, &S, BK);
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

// ---- grouped weight gradients: two products with the same K (tokens) in ONE ping-pong launch.
// The split count is chosen for the pair: the estimated makespan ceil(T S / CUs) * ceil(nk / S) K-tiles
// plus the slab traffic of S > 1 (written once, read once by slab_reduce_kernel, ~5 TB/s), in units of
// one K-tile of one workgroup (~1.8 us at the measured 1.2 PF/s).
// Split count of the grouped launch, or 0 when the pair cannot be grouped (then call nd_wgrad twice).
// Slab workspace: S * M0 * N0 floats for product 0 and S * M1 * N1 for product 1 (S > 1).
ND_API int nd_wgrad2_splits(int M0, int N0, int M1, int N1, int K) {
  const char* ev = wgrad_env();
  if ((ev && ev[0]) || !wgrad_pp_eligible(M0, N0, K, 8, 8, 4) || !wgrad_pp_eligible(M1, N1, K, 8, 8, 4)) return 0;
  const int T0 = ((M0 + 255) / 256) * ((N0 + 255) / 256), T1 = ((M1 + 255) / 256) * ((N1 + 255) / 256);
  const int64_t mn = (int64_t)M0 * N0 + (int64_t)M1 * N1;
  const int S = group_splits(T0 + T1, K, mn);
  // group only when the model predicts a clear win over the two separate launches (each with its own plan):
  // Llama-150M down + gate|up 1039 vs 1114 K-tile units (grouped); Llama-1B 1241 vs 1208 (separate)
  int S0, S1;
  plan(M0, N0, K, &S0);
  plan(M1, N1, K, &S1);
  const double sep = split_cost(T0, K, (int64_t)M0 * N0, S0) + split_cost(T1, K, (int64_t)M1 * N1, S1);
  return split_cost(T0 + T1, K, mn, S) < 0.97 * sep ? S : 0;
}

ND_API int nd_wgrad2(const void* A0, const void* B0, float* C0, float* slab0, int M0, int N0, int64_t lda0, int64_t ldb0,
                     int64_t ldc0, const void* A1, const void* B1, float* C1, float* slab1, int M1, int N1, int64_t lda1,
                     int64_t ldb1, int64_t ldc1, int K, hipStream_t s) {
  int S = nd_wgrad2_splits(M0, N0, M1, N1, K);
  if (S <= 0 || !wgrad_pp_eligible(M0, N0, K, lda0, ldb0, ldc0) || !wgrad_pp_eligible(M1, N1, K, lda1, ldb1, ldc1))
    return (int)hipErrorInvalidValue;
  if (S > 1 && (slab0 == nullptr || slab1 == nullptr)) return (int)hipErrorInvalidValue;
  const int kchunk = fit_kchunk(K, &S, 64);  // may only lower S: the caller's slabs stay large enough
  const int T0 = ((M0 + 255) / 256) * ((N0 + 255) / 256), T1 = ((M1 + 255) / 256) * ((N1 + 255) / 256);
  const size_t lds = 2 * (size_t)WPP_BUF_B;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad_pp_kernel<true>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return (int)attr;
  const WgProb p0{(const bf16_t*)A0, (const bf16_t*)B0, C0, slab0, M0, N0, lda0, ldb0, ldc0};
  const WgProb p1{(const bf16_t*)A1, (const bf16_t*)B1, C1, slab1, M1, N1, lda1, ldb1, ldc1};
  hipLaunchKernelGGL(wgrad_pp_kernel<true>, dim3((T0 + T1) * S), dim3(512), lds, s, p0, p1, T0 * S, K, S, kchunk);
  if (S > 1) {
    const WgProb* ps[2] = {&p0, &p1};
    for (const WgProb* p : ps) {
      int64_t blocks = ((int64_t)p->M * p->N / 4 + 255) / 256;
      if (blocks > 4096) blocks = 4096;
      hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p->slab, p->C, p->M, p->N, p->ldc,
                         S);
    }
  }
  ND_LAUNCH_CHECK();
}

// fp8 weight gradient: C[M, N] (fp32) += sa sb A^T B with A = dY8 [K, M] (lda bytes; fa 0 e4m3, 1 e5m2),
// B = X8 [K, N] (ldb bytes, e4m3).  K % 128 == 0, M, N % 16 == 0, lda / ldb % 16 == 0.  Slab workspace as
// nd_wgrad (nd_wgrad_splits(M, N, K) planes).
ND_API int nd_wgrad_f8(const void* A, const void* B, float* C, float* slab, int M, int N, int K, int64_t lda,
                       int64_t ldb, int64_t ldc, const float* sa, const float* sb, int fa, hipStream_t s) {
  if (M % 16 || N % 16 || lda % 16 || ldb % 16 || ldc % 4 || K % 128 || K <= 0 || M < 256 || N < 256 || !sa || !sb ||
      (fa != 0 && fa != 1) || (int64_t)128 * (lda > ldb ? lda : ldb) >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  int S;
  plan(M, N, K, &S, false);
  if (S > 1 && slab == nullptr) return (int)hipErrorInvalidValue;
  const int kchunk = fit_kchunk(K, &S, 128);
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  const size_t lds = 2 * (size_t)W8_BUF_B;  // 128 KiB
  static const hipError_t attr =
      (hipError_t)(hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad8_pp_kernel<0>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) |
                   hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad8_pp_kernel<1>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  if (attr != hipSuccess) return (int)attr;
  if (fa == 0)
    hipLaunchKernelGGL(wgrad8_pp_kernel<0>, dim3(tiles * S), dim3(512), lds, s, (const uint8_t*)A, (const uint8_t*)B, C,
                       slab, M, N, K, lda, ldb, ldc, S, kchunk, sa, sb);
  else
    hipLaunchKernelGGL(wgrad8_pp_kernel<1>, dim3(tiles * S), dim3(512), lds, s, (const uint8_t*)A, (const uint8_t*)B, C,
                       slab, M, N, K, lda, ldb, ldc, S, kchunk, sa, sb);
  if (S > 1) {
    int64_t blocks = ((int64_t)M * N / 4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, s, slab, C, M, N, ldc, S);
  }
  ND_LAUNCH_CHECK();
}
