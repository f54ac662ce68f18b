// Forward-projection GEMM for gfx950:  C[M, N] (bf16) = A[M, K] . B[N, K]^T   (both operands
// K-contiguous: activations x [tokens, in] and a weight W [out, in], the nn.Linear layout).
//
// 256 x 256 tile per 512-thread workgroup (8 waves as 2 (M) x 4 (N), 128 x 64 per wave = 8 x 4
// v_mfma_f32_16x16x32_bf16 tiles), BK = 64, two LDS stages of 2 x 32 KiB filled by LDS-DMA
// (global_load_lds_dwordx4 from inline asm, scalar base + per-lane offsets fixed per kernel).
// K-major tiles ([row][64 k], 128-B rows) are read straight into MFMA fragments with ds_read_b128
// (lane l: row l & 15, k-chunk l >> 4); the 16-B chunk index is XOR-swizzled with (row >> 1) & 7,
// which spreads every ds_read_b128 lane group over 16 distinct bank slots (conflict-free), applied
// on the DMA source address so the LDS image stays lane-linear.  The MFMA is issued as B . A^T so
// each lane ends with 4 consecutive output columns of one row -> one 8-B bf16 store per tile.
// XCD-aware workgroup order keeps the workgroups that share an A row-panel on one L2.
#include "common.h"

using namespace nd;

namespace {
typedef __bf16 bfv8 __attribute__((ext_vector_type(8)));
constexpr int TM = 256, TN = 256, TK = 64;

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bfv8, a), __builtin_bit_cast(bfv8, b), c, 0, 0, 0);
}

__device__ __forceinline__ void glds(const void* sbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds) : "memory");
}

// element offset of (row, k) in a [256][64] K-major tile
__device__ __forceinline__ int koff(int row, int k) { return row * 64 + ((((k >> 3) ^ ((row >> 1) & 7))) << 3) + (k & 7); }

// DMA plan of one 256 x 64 K-major operand tile: 32 wave-instructions of 8 rows x 128 B; wave w
// issues instructions w, w+8, w+16, w+24 (rows 8 ins .. 8 ins + 7).
struct KDma {
  uint32_t voff[4];
  __device__ __forceinline__ void init(int64_t ld, int r0, int rows) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int row = 8 * (w + 8 * it) + (lane >> 3);
      const int lch = (lane & 7) ^ ((row >> 1) & 7);
      int gr = r0 + row;
      gr = gr < rows ? gr : rows - 1;  // tail rows: any valid row (their outputs are never stored)
      voff[it] = (uint32_t)(((int64_t)(gr - r0) * ld + lch * 8) * 2);
    }
  }
  __device__ __forceinline__ void issue(const bf16_t* base, uint32_t lds_tile) const {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int it = 0; it < 4; ++it) glds(base, voff[it], lds_tile + (uint32_t)((w + 8 * it) * 1024));
  }
};
}  // namespace

// STAMP (diagnostic build only): per wave, cycles spent in the tile-boundary wait (vmcnt + barrier),
// in the LDS-read waits, and in total, written to dbg[4 * (block * 8 + wave)] (+ elapsed 100-MHz ticks).
template <bool STAMP>
__global__ void __launch_bounds__(512, 2) gemm_nt_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                         bf16_t* __restrict__ C, int M, int N, int K, int64_t lda,
                                                         int64_t ldb, int64_t ldc, uint64_t* __restrict__ dbg) {
  uint64_t t_start = 0, t_wait = 0, t_lds = 0, r_start = 0;
  if (STAMP) { t_start = __builtin_amdgcn_s_memtime(); r_start = __builtin_amdgcn_s_memrealtime(); }
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];  // [stage][A 256x64 | B 256x64]
  constexpr int TE = TM * TK;                                    // elements per operand tile
  const int tn = (N + TN - 1) / TN, tiles = ((M + TM - 1) / TM) * tn;
  const int id = xcd_remap(blockIdx.x, tiles);
  const int m0 = (id / tn) * TM, n0 = (id % tn) * TN;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = w >> 2, wn = w & 3;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) bf16_t*)smem);

  KDma da, db;
  da.init(lda, m0, M);
  db.init(ldb, n0, N);
  const bf16_t* Ab = A + (int64_t)m0 * lda;
  const bf16_t* Bb = B + (int64_t)n0 * ldb;
  auto stage = [&](int kt) {
    const uint32_t t = lds0 + (uint32_t)((kt & 1) * 2 * TE * 2);
    da.issue(Ab + kt * TK, t);
    db.issue(Bb + kt * TK, t + TE * 2);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / TK;
  stage(0);
  for (int kt = 0; kt < nk; ++kt) {
    uint64_t t0 = 0;
    if (STAMP) t0 = __builtin_amdgcn_s_memtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's part of tile kt has landed
    __builtin_amdgcn_s_barrier();                     // everyone's; buffer (kt+1)&1 is free again
    if (STAMP) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); t_wait += __builtin_amdgcn_s_memtime() - t0; }
    if (kt + 1 < nk) stage(kt + 1);
    const bf16_t* at = smem + (kt & 1) * 2 * TE;
    const bf16_t* bt = at + TE;
#pragma unroll
    for (int ks = 0; ks < TK / 32; ++ks) {
      const int kc = ks * 32 + (lane >> 4) * 8;
      bf16x8 fa[8], fb[4];
#pragma unroll
      for (int b = 0; b < 4; ++b)
        fb[b] = *reinterpret_cast<const bf16x8*>(&bt[koff(wn * 64 + b * 16 + (lane & 15), kc)]);
#pragma unroll
      for (int a = 0; a < 8; ++a)
        fa[a] = *reinterpret_cast<const bf16x8*>(&at[koff(wm * 128 + a * 16 + (lane & 15), kc)]);
      if (STAMP) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        t_lds += __builtin_amdgcn_s_memtime() - t1;
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = mfma16(fb[b], fa[a], acc[a][b]);  // C^T tile: lane = row m
      __builtin_amdgcn_s_setprio(0);
    }
  }
  // acc[a][b] lane l reg r: C[m0 + wm*128 + a*16 + (l & 15)][n0 + wn*64 + b*16 + 4 (l >> 4) + r]
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int m = m0 + wm * 128 + a * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int n = n0 + wn * 64 + b * 16 + 4 * (lane >> 4);
      if (n >= N) continue;
      uint2 v;
      v.x = pack2(acc[a][b][0], acc[a][b][1]);
      v.y = pack2(acc[a][b][2], acc[a][b][3]);
      *reinterpret_cast<uint2*>(C + (int64_t)m * ldc + n) = v;
    }
  }
  if (STAMP && lane == 0) {
    uint64_t* d = dbg + 4 * ((int64_t)blockIdx.x * 8 + w);
    d[0] = t_wait;
    d[1] = t_lds;
    d[2] = __builtin_amdgcn_s_memtime() - t_start;
    d[3] = __builtin_amdgcn_s_memrealtime() - r_start;  // 100 MHz
  }
}



// C[M, N] = A[M, K] . B[N, K]^T (bf16 in / bf16 out, fp32 accumulate).  K % 64 == 0, N % 4 == 0,
// lda / ldb % 8 == 0, ldc % 4 == 0.
ND_API int nd_gemm_nt(const void* A, const void* B, void* C, int M, int N, int K, int64_t lda, int64_t ldb,
                      int64_t ldc, uint64_t* dbg, hipStream_t s) {
  if (K % TK || N % 4 || lda % 8 || ldb % 8 || ldc % 4 || M <= 0 || N <= 0) return (int)hipErrorInvalidValue;
  const int tiles = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  const size_t lds = 2 * 2 * (size_t)TM * TK * sizeof(bf16_t);  // 128 KiB
  static const hipError_t attr_ok =
      (hipError_t)(hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<false>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) |
                   hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_kernel<true>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  (void)attr_ok;
  if (dbg)
    hipLaunchKernelGGL(gemm_nt_kernel<true>, dim3(tiles), dim3(512), lds, s, (const bf16_t*)A, (const bf16_t*)B,
                       (bf16_t*)C, M, N, K, lda, ldb, ldc, dbg);
  else
    hipLaunchKernelGGL(gemm_nt_kernel<false>, dim3(tiles), dim3(512), lds, s, (const bf16_t*)A, (const bf16_t*)B,
                       (bf16_t*)C, M, N, K, lda, ldb, ldc, dbg);
  ND_LAUNCH_CHECK();
}
