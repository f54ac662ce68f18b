// fp8 quantisation for the fp8 inner step (BASELINE config 5): one streaming pass that scales,
// saturates and converts to OCP fp8 (gfx950 v_cvt_pk_fp8_f32 / v_cvt_pk_bf8_f32: e4m3fn / e5m2,
// round-to-nearest-even) AND records amax(|x|) for the delayed-scaling recipe.
//   out[i] = fp8(clamp(x[i] * scale, -FMAX, FMAX)),   amax_out = max(amax_out, max |x|)
// The scale is read from device memory (no host sync).  8 elements per thread: 16-B bf16 loads,
// 8-B fp8 stores; amax reduced per block, then one atomicMax (float as ordered int bits) per block
// into one of `amax_parts` partial slots (blockIdx % parts): a single hot address serialises the
// atomics in L2 (measured 160-200 us per 32M-element cast with one slot and per-wave atomics, vs
// ~15 us of streaming); the recipe reduces the partials once per inner step.
#include "common.h"

using namespace nd;

// cvt4 (saturating OCP fp8 conversion of 4 floats): common.h

template <int XDT, int FMT>
__global__ void __launch_bounds__(256) fp8_cast_kernel(const void* __restrict__ x, int64_t n,
                                                       const float* __restrict__ scale_p, uint8_t* __restrict__ out,
                                                       float* __restrict__ amax_out, int amax_parts) {
  const float scale = scale_p ? scale_p[0] : 1.f;
  float amax = 0.f;
  const int64_t n8 = n >> 3;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    Vec8<XDT>::load(x, i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[j]));
    if (out) {  // out == nullptr: amax-only pass (weights use current scaling: amax first, then cast)
      uint2 o;
      o.x = cvt4<FMT>(v[0] * scale, v[1] * scale, v[2] * scale, v[3] * scale);
      o.y = cvt4<FMT>(v[4] * scale, v[5] * scale, v[6] * scale, v[7] * scale);
      *reinterpret_cast<uint2*>(out + i * 8) = o;
    }
  }
  for (int64_t i = n8 * 8 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float f = XDT == BF16 ? bf2f(reinterpret_cast<const bf16_t*>(x)[i]) : reinterpret_cast<const float*>(x)[i];
    amax = fmaxf(amax, fabsf(f));
    if (out) out[i] = (uint8_t)(cvt4<FMT>(f * scale, 0.f, 0.f, 0.f) & 0xff);
  }
  if (amax_out) {
    __shared__ float red[4];
    amax = wave_max(amax);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
    __syncthreads();
    if (threadIdx.x == 0) {
      amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
      // non-negative floats order like their int bit patterns
      atomicMax(reinterpret_cast<int*>(amax_out + blockIdx.x % amax_parts), __float_as_int(amax));
    }
  }
}

ND_API int nd_fp8_cast(const void* x, int xdt, int64_t n, const float* scale, void* out, int fmt, float* amax_out,
                       int amax_parts, hipStream_t s) {
  int64_t blocks = (n / 8 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;  // 8 blocks/CU, grid-stride beyond
  if (amax_parts < 1) amax_parts = 1;
  const dim3 g((unsigned)blocks), b(256);
  uint8_t* o = (uint8_t*)out;
  if (xdt == BF16) {
    if (fmt == 0) hipLaunchKernelGGL((fp8_cast_kernel<BF16, 0>), g, b, 0, s, x, n, scale, o, amax_out, amax_parts);
    else hipLaunchKernelGGL((fp8_cast_kernel<BF16, 1>), g, b, 0, s, x, n, scale, o, amax_out, amax_parts);
  } else {
    if (fmt == 0) hipLaunchKernelGGL((fp8_cast_kernel<F32, 0>), g, b, 0, s, x, n, scale, o, amax_out, amax_parts);
    else hipLaunchKernelGGL((fp8_cast_kernel<F32, 1>), g, b, 0, s, x, n, scale, o, amax_out, amax_parts);
  }
  ND_LAUNCH_CHECK();
}

// Cast + transpose in one pass (fp8 weight-gradient GEMM operands): x [rows, cols] (row stride ld)
// -> out [rows, cols] (optional, row-major) and outT [cols, rows] (row-major), both fp8(x * scale),
// plus amax.  64 x 64 tile per 256-thread block: each thread loads 2 x 8 consecutive elements
// (16-B bf16 loads), writes them straight to `out`, and parks the fp8 bytes in LDS; the transposed
// tile is then written as 16-B rows of outT (16 consecutive source rows of one column per thread).
// rows and cols must be multiples of 64 (checked by the caller).
template <int XDT, int FMT>
__global__ void __launch_bounds__(256) fp8_cast_t_kernel(const void* __restrict__ x, int rows, int cols, int64_t ld,
                                                         const float* __restrict__ scale_p, uint8_t* __restrict__ out,
                                                         uint8_t* __restrict__ outT, float* __restrict__ amax_out,
                                                         int amax_parts) {
  __shared__ uint8_t tile[64][64 + 16];
  const float scale = scale_p ? scale_p[0] : 1.f;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int t = threadIdx.x;
  float amax = 0.f;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = t + it * 256;          // 512 vectors of 8 elements
    const int r = idx >> 3, cv = (idx & 7) * 8;
    float v[8];
    Vec8<XDT>::load(x, (int64_t)(r0 + r) * ld + c0 + cv, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[j]));
    uint2 o;
    o.x = cvt4<FMT>(v[0] * scale, v[1] * scale, v[2] * scale, v[3] * scale);
    o.y = cvt4<FMT>(v[4] * scale, v[5] * scale, v[6] * scale, v[7] * scale);
    if (out) *reinterpret_cast<uint2*>(out + (int64_t)(r0 + r) * cols + c0 + cv) = o;
    *reinterpret_cast<uint2*>(&tile[r][cv]) = o;
  }
  __syncthreads();
  {
    const int c = t >> 2, rq = (t & 3) * 16;  // column c, source rows rq .. rq+15
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      w[q] = (uint32_t)tile[rq + 4 * q][c] | ((uint32_t)tile[rq + 4 * q + 1][c] << 8) |
             ((uint32_t)tile[rq + 4 * q + 2][c] << 16) | ((uint32_t)tile[rq + 4 * q + 3][c] << 24);
    }
    *reinterpret_cast<uint4*>(outT + (int64_t)(c0 + c) * rows + r0 + rq) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  if (amax_out) {
    __shared__ float red[4];
    amax = wave_max(amax);
    if ((t & 63) == 0) red[t >> 6] = amax;
    __syncthreads();
    if (t == 0) {
      amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
      const int b = blockIdx.y * gridDim.x + blockIdx.x;
      atomicMax(reinterpret_cast<int*>(amax_out + b % amax_parts), __float_as_int(amax));
    }
  }
}

ND_API int nd_fp8_cast_t(const void* x, int xdt, int rows, int cols, int64_t ld, const float* scale, void* out,
                         void* outT, int fmt, float* amax_out, int amax_parts, hipStream_t s) {
  if (rows % 64 || cols % 64 || ld % 8 || outT == nullptr) return (int)hipErrorInvalidValue;
  if (amax_parts < 1) amax_parts = 1;
  const dim3 g(cols / 64, rows / 64), b(256);
  uint8_t *o = (uint8_t*)out, *oT = (uint8_t*)outT;
  if (xdt == BF16) {
    if (fmt == 0) hipLaunchKernelGGL((fp8_cast_t_kernel<BF16, 0>), g, b, 0, s, x, rows, cols, ld, scale, o, oT, amax_out, amax_parts);
    else hipLaunchKernelGGL((fp8_cast_t_kernel<BF16, 1>), g, b, 0, s, x, rows, cols, ld, scale, o, oT, amax_out, amax_parts);
  } else {
    if (fmt == 0) hipLaunchKernelGGL((fp8_cast_t_kernel<F32, 0>), g, b, 0, s, x, rows, cols, ld, scale, o, oT, amax_out, amax_parts);
    else hipLaunchKernelGGL((fp8_cast_t_kernel<F32, 1>), g, b, 0, s, x, rows, cols, ld, scale, o, oT, amax_out, amax_parts);
  }
  ND_LAUNCH_CHECK();
}
