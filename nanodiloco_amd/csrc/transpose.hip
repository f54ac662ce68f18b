// bf16 matrix transpose for the W^T copies the input-gradient GEMMs read (ops/linear.py):
// dst[c][r] = src[r][c].  Refreshed once per optimizer step for every projection weight, so it
// only has to be HBM-bound rather than the strided-copy rate of a generic copy_(w.t()).
//
// One 256-thread workgroup per 64 x 64 tile: each thread loads two 16-B row chunks (coalesced
// 128-B row segments), the tile goes through LDS with a 2-element row pad (odd 32-bit stride, so
// the column walk of the write-out hits distinct banks), and each thread emits two 16-B chunks of
// transposed rows.  Edge tiles are guarded element-wise; rows / cols need not be multiples of 64.
#include "common.h"

using namespace nd;

namespace {
constexpr int TT = 64, PAD = 2;

template <bool VEC>  // VEC: 16-B aligned bases and strides (vector path for full tiles)
__global__ void __launch_bounds__(256) transpose_bf16_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                             int rows, int cols, int64_t lds, int64_t ldd) {
  __shared__ bf16_t tile[TT][TT + PAD];
  const int tc = (cols + TT - 1) / TT;
  const int r0 = (blockIdx.x / tc) * TT, c0 = (blockIdx.x % tc) * TT;
  const bool full = VEC && (r0 + TT <= rows) && (c0 + TT <= cols);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = threadIdx.x + it * 256;  // 512 chunks of 8 elements
    const int r = idx >> 3, ch = idx & 7;
    const int gr = r0 + r, gc = c0 + ch * 8;
    if (full) {
      const uint4 v = *reinterpret_cast<const uint4*>(src + (int64_t)gr * lds + gc);
      const bf16_t* e = reinterpret_cast<const bf16_t*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) tile[r][ch * 8 + j] = e[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        tile[r][ch * 8 + j] = (gr < rows && gc + j < cols) ? src[(int64_t)gr * lds + gc + j] : (bf16_t)0;
    }
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = threadIdx.x + it * 256;
    const int c = idx >> 3, ch = idx & 7;  // output row = source column c0 + c
    const int orow = c0 + c, ocol = r0 + ch * 8;
    uint4 v;
    bf16_t* e = reinterpret_cast<bf16_t*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = tile[ch * 8 + j][c];
    if (full) {
      *reinterpret_cast<uint4*>(dst + (int64_t)orow * ldd + ocol) = v;
    } else if (orow < cols) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (ocol + j < rows) dst[(int64_t)orow * ldd + ocol + j] = e[j];
    }
  }
}
}  // namespace

// dst [cols, rows] (row stride ldd) = src [rows, cols] (row stride lds) ^T.  Full tiles use 16-B
// vector accesses when both bases are 16-B aligned and both strides are multiples of 8 elements.
ND_API int nd_transpose_bf16(const void* src, void* dst, int rows, int cols, int64_t lds, int64_t ldd,
                             hipStream_t s) {
  if (rows <= 0 || cols <= 0 || lds < cols || ldd < rows) return (int)hipErrorInvalidValue;
  const bool vec = !(lds % 8 || ldd % 8 || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15));
  const int64_t tiles = (int64_t)((rows + TT - 1) / TT) * ((cols + TT - 1) / TT);
  if (vec)
    hipLaunchKernelGGL(transpose_bf16_kernel<true>, dim3((unsigned)tiles), dim3(256), 0, s, (const bf16_t*)src,
                       (bf16_t*)dst, rows, cols, lds, ldd);
  else
    hipLaunchKernelGGL(transpose_bf16_kernel<false>, dim3((unsigned)tiles), dim3(256), 0, s, (const bf16_t*)src,
                       (bf16_t*)dst, rows, cols, lds, ldd);
  ND_LAUNCH_CHECK();
}
