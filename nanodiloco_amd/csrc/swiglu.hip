// SwiGLU on the fused gate|up GEMM output (K7).  gu: [n, 2F] (gate cols [0,F), up cols [F,2F)).
//   fwd: act = silu(g) * u                      -> [n, F]
//   bwd: dg = dy * u * s * (1 + g * (1 - s)),  du = dy * silu(g)   -> d(gu) [n, 2F]
// Memory-bound; 8 elements per thread with 16-B bf16 vector accesses, fp32 math.
// Q: fused fp8 side output for the fp8 inner step (common.h Fp8Out): act8 = e4m3 of the activation
// (the down projection's operand), d(gu)8 = e5m2 of the gradient (the gate|up dgrad operand),
// written by the same pass instead of a separate cast over the bf16 tensor (3 B/elem -> 1 B/elem).
#include "common.h"

using namespace nd;

__device__ __forceinline__ float sigm(float x) { return fast_sigmoid(x); }

template <int DT, bool Q = false>
__global__ void __launch_bounds__(256) swiglu_fwd_kernel(const void* __restrict__ gu, void* __restrict__ out,
                                                         int64_t n, int F, Fp8Out q8) {
  const int f8 = F >> 3;
  const int64_t total = n * f8;
  float amax = 0.f;
  const float qsc = Q ? q8.scale[0] : 1.f;
  for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < total; it += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = it / f8;
    const int c = (int)(it % f8) * 8;
    float g[8], u[8], o[8];
    Vec8<DT>::load(gu, r * 2 * F + c, g);
    Vec8<DT>::load(gu, r * 2 * F + F + c, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] * sigm(g[j]) * u[j];
    if (Q) put8_bf16_q(out, r * F + c, o, q8, qsc, amax);  // DT == BF16 (launcher)
    else Vec8<DT>::store(out, r * F + c, o);
  }
  if (Q) block_amax_commit<256>(amax, q8.amax, q8.parts);
}

template <int DT, bool Q = false>
__global__ void __launch_bounds__(256) swiglu_bwd_kernel(const void* __restrict__ dy, const void* __restrict__ gu,
                                                         void* __restrict__ dgu, int64_t n, int F, Fp8Out q8) {
  const int f8 = F >> 3;
  const int64_t total = n * f8;
  float amax = 0.f;
  const float qsc = Q ? q8.scale[0] : 1.f;
  for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < total; it += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = it / f8;
    const int c = (int)(it % f8) * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    Vec8<DT>::load(gu, r * 2 * F + c, g);
    Vec8<DT>::load(gu, r * 2 * F + F + c, u);
    Vec8<DT>::load(dy, r * F + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = sigm(g[j]);
      du[j] = d[j] * g[j] * s;
      dg[j] = d[j] * u[j] * s * (1.f + g[j] * (1.f - s));
    }
    if (Q) {  // DT == BF16 (launcher)
      put8_bf16_q(dgu, r * 2 * F + c, dg, q8, qsc, amax);
      put8_bf16_q(dgu, r * 2 * F + F + c, du, q8, qsc, amax);
    } else {
      Vec8<DT>::store(dgu, r * 2 * F + c, dg);
      Vec8<DT>::store(dgu, r * 2 * F + F + c, du);
    }
  }
  if (Q) block_amax_commit<256>(amax, q8.amax, q8.parts);
}

static unsigned grid_for(int64_t total) {
  int64_t b = (total + 255) / 256;
  return (unsigned)(b > 16384 ? 16384 : (b < 1 ? 1 : b));
}

ND_API int nd_swiglu_fwd(const void* gu, void* out, int dt, int64_t n, int F, hipStream_t s) {
  if (F % 8) return (int)hipErrorInvalidValue;
  const unsigned g = grid_for(n * (F / 8));
  const Fp8Out none{nullptr, nullptr, nullptr, 1, 0};
  if (dt == BF16) hipLaunchKernelGGL(swiglu_fwd_kernel<BF16>, dim3(g), dim3(256), 0, s, gu, out, n, F, none);
  else hipLaunchKernelGGL(swiglu_fwd_kernel<F32>, dim3(g), dim3(256), 0, s, gu, out, n, F, none);
  ND_LAUNCH_CHECK();
}

ND_API int nd_swiglu_bwd(const void* dy, const void* gu, void* dgu, int dt, int64_t n, int F, hipStream_t s) {
  if (F % 8) return (int)hipErrorInvalidValue;
  const unsigned g = grid_for(n * (F / 8));
  const Fp8Out none{nullptr, nullptr, nullptr, 1, 0};
  if (dt == BF16) hipLaunchKernelGGL(swiglu_bwd_kernel<BF16>, dim3(g), dim3(256), 0, s, dy, gu, dgu, n, F, none);
  else hipLaunchKernelGGL(swiglu_bwd_kernel<F32>, dim3(g), dim3(256), 0, s, dy, gu, dgu, n, F, none);
  ND_LAUNCH_CHECK();
}

// bf16 variants with the fused fp8 side output (q: [n, F] fwd / [n, 2F] bwd fp8 bytes)
ND_API int nd_swiglu_fwd_q(const void* gu, void* out, int64_t n, int F, void* q, const float* scale, float* amax,
                           int parts, int fmt, hipStream_t s) {
  if (F % 8 || !q || !scale || !amax || parts < 1) return (int)hipErrorInvalidValue;
  const Fp8Out q8{(uint8_t*)q, scale, amax, parts, fmt};
  hipLaunchKernelGGL((swiglu_fwd_kernel<BF16, true>), dim3(grid_for(n * (F / 8))), dim3(256), 0, s, gu, out, n, F, q8);
  ND_LAUNCH_CHECK();
}

ND_API int nd_swiglu_bwd_q(const void* dy, const void* gu, void* dgu, int64_t n, int F, void* q, const float* scale,
                           float* amax, int parts, int fmt, hipStream_t s) {
  if (F % 8 || !q || !scale || !amax || parts < 1) return (int)hipErrorInvalidValue;
  const Fp8Out q8{(uint8_t*)q, scale, amax, parts, fmt};
  hipLaunchKernelGGL((swiglu_bwd_kernel<BF16, true>), dim3(grid_for(n * (F / 8))), dim3(256), 0, s, dy, gu, dgu, n, F,
                     q8);
  ND_LAUNCH_CHECK();
}
