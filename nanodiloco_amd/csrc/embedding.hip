// Token embedding gather / scatter-add (K1) on fp32 tables.
//   fwd: out[i, :] = W[ids[i], :]        one wave per row, 16-B loads/stores
//   bwd: gW[ids[i], :] += dy[i, :]       one wave per row, each wave-instruction = 64 f32 atomics on
//                                        256 contiguous bytes (full-rate atomic shape on MI355X)
// Out-of-range ids are skipped (fwd writes zeros) instead of faulting the device.
#include "common.h"

using namespace nd;

__global__ void __launch_bounds__(256) embed_fwd_kernel(const int64_t* __restrict__ ids, const float* __restrict__ W,
                                                        float* __restrict__ out, int64_t n, int d, int V) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int64_t r = wave; r < n; r += (int64_t)gridDim.x * 4) {
    const int64_t id = ids[r];
    const bool ok = id >= 0 && id < V;
    for (int c = lane * 4; c < d; c += 256) {
      float4 v = ok ? *reinterpret_cast<const float4*>(W + id * d + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(out + r * d + c) = v;
    }
  }
}

__global__ void __launch_bounds__(256) embed_bwd_kernel(const int64_t* __restrict__ ids, const float* __restrict__ dy,
                                                        float* __restrict__ gW, int64_t n, int d, int V) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int64_t r = wave; r < n; r += (int64_t)gridDim.x * 4) {
    const int64_t id = ids[r];
    if (id < 0 || id >= V) continue;
    for (int c = lane; c < d; c += 64) atomicAdd(gW + id * d + c, dy[r * d + c]);
  }
}

ND_API int nd_embedding_fwd(const int64_t* ids, const float* W, float* out, int64_t n, int d, int V, hipStream_t s) {
  if (d % 4) return (int)hipErrorInvalidValue;
  int64_t blocks = (n + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ids, W, out, n, d, V);
  ND_LAUNCH_CHECK();
}

ND_API int nd_embedding_bwd(const int64_t* ids, const float* dy, float* gW, int64_t n, int d, int V, hipStream_t s) {
  int64_t blocks = (n + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ids, dy, gW, n, d, V);
  ND_LAUNCH_CHECK();
}
