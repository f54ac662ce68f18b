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

// Deterministic backward: rows visited in sorted-id order (sid = ids[perm], perm a STABLE argsort), one
// wave per run of equal ids summing its dy rows in position order, then one plain read-add-write of
// the table row -- bitwise reproducible (the atomic kernel's float adds land in arrival order).
__global__ void __launch_bounds__(256) embed_bwd_sorted_kernel(const int64_t* __restrict__ sid,
                                                               const int64_t* __restrict__ perm,
                                                               const float* __restrict__ dy, float* __restrict__ gW,
                                                               int64_t n, int d, int V) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int64_t r = wave; r < n; r += (int64_t)gridDim.x * 4) {
    const int64_t id = sid[r];
    if ((r > 0 && sid[r - 1] == id) || id < 0 || id >= V) continue;  // not the start of a run
    int64_t e = r + 1;
    while (e < n && sid[e] == id) ++e;
    for (int c = lane * 4; c < d; c += 256) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int64_t j = r; j < e; ++j) {
        const float4 v = *reinterpret_cast<const float4*>(dy + perm[j] * d + c);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      float4* g = reinterpret_cast<float4*>(gW + id * d + c);
      float4 o = *g;
      o.x += acc.x; o.y += acc.y; o.z += acc.z; o.w += acc.w;
      *g = o;
    }
  }
}

ND_API int nd_embedding_bwd_sorted(const int64_t* sid, const int64_t* perm, const float* dy, float* gW, int64_t n,
                                   int d, int V, hipStream_t s) {
  if (d % 4) return (int)hipErrorInvalidValue;
  int64_t blocks = (n + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(embed_bwd_sorted_kernel, dim3((unsigned)blocks), dim3(256), 0, s, sid, perm, dy, gW, n, d, V);
  ND_LAUNCH_CHECK();
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
