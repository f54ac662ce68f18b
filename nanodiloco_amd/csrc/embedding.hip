// Token embedding gather / scatter-add (K1) on fp32 tables.
//   fwd: out[i, :] = W[ids[i], :]        one wave per row, 16-B loads/stores; out fp32, or bf16 (RNE) for the
//                                        bf16 residual stream (then dy of the backward is bf16 too)
//   bwd: gW[ids[i], :] += dy[i, :]       one wave per row, each wave-instruction = 64 f32 atomics on
//                                        256 contiguous bytes (full-rate atomic shape on MI355X)
// Out-of-range ids are skipped (fwd writes zeros) instead of faulting the device.
#include "common.h"

using namespace nd;

__device__ __forceinline__ void put4(float* out, int64_t i, float4 v) { *reinterpret_cast<float4*>(out + i) = v; }
__device__ __forceinline__ void put4(bf16_t* out, int64_t i, float4 v) {
  *reinterpret_cast<uint2*>(out + i) = make_uint2(pack2(v.x, v.y), pack2(v.z, v.w));
}
__device__ __forceinline__ float4 get4(const float* p, int64_t i) { return *reinterpret_cast<const float4*>(p + i); }
__device__ __forceinline__ float4 get4(const bf16_t* p, int64_t i) {
  const uint2 u = *reinterpret_cast<const uint2*>(p + i);
  return make_float4(lo_bf(u.x), hi_bf(u.x), lo_bf(u.y), hi_bf(u.y));
}
__device__ __forceinline__ float get1(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float get1(const bf16_t* p, int64_t i) { return bf2f(p[i]); }

template <typename OT>
__global__ void __launch_bounds__(256) embed_fwd_kernel(const int64_t* __restrict__ ids, const float* __restrict__ W,
                                                        OT* __restrict__ out, int64_t n, int d, int V) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int64_t r = wave; r < n; r += (int64_t)gridDim.x * 4) {
    const int64_t id = ids[r];
    const bool ok = id >= 0 && id < V;
    for (int c = lane * 4; c < d; c += 256) {
      float4 v = ok ? *reinterpret_cast<const float4*>(W + id * d + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      put4(out, r * d + c, v);
    }
  }
}

template <typename DT>
__global__ void __launch_bounds__(256) embed_bwd_kernel(const int64_t* __restrict__ ids, const DT* __restrict__ dy,
                                                        float* __restrict__ gW, int64_t n, int d, int V) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  for (int64_t r = wave; r < n; r += (int64_t)gridDim.x * 4) {
    const int64_t id = ids[r];
    if (id < 0 || id >= V) continue;
    for (int c = lane; c < d; c += 64) atomicAdd(gW + id * d + c, get1(dy, r * d + c));
  }
}

// Deterministic backward over the sorted ids (sid = ids[perm], perm a STABLE argsort): every table row
// is summed in position order and added with one plain read-add-write -- bitwise reproducible (the
// atomic kernel's float adds land in arrival order).  Work is split into fixed 64-row chunks of the
// sorted order so that a long run of one id (thousands of pad rows in a left-padded HF micro-batch)
// does not serialise on one wave:
//   pass 1 (one wave per chunk): runs that start and end inside the chunk go straight to gW; the
//     chunk's first segment, when it continues a run from the previous chunk, is written to
//     head[chunk]; its last segment, when it starts a run that continues past the chunk, to tail[chunk].
//   pass 2 (one wave per chunk that owns such a crossing run): tail[c] + head[c+1] + head[c+2] + ...
//     in chunk order, then one read-add-write of the table row.
constexpr int kEmbChunk = 64;

template <typename DT>
__global__ void __launch_bounds__(256) embed_bwd_sorted_chunks_kernel(const int64_t* __restrict__ sid,
                                                                      const int64_t* __restrict__ perm,
                                                                      const DT* __restrict__ dy,
                                                                      float* __restrict__ gW, float* __restrict__ head,
                                                                      float* __restrict__ tail, int64_t n, int d, int V) {
  const int lane = threadIdx.x & 63;
  const int64_t nchunks = (n + kEmbChunk - 1) / kEmbChunk;
  for (int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < nchunks; c += (int64_t)gridDim.x * 4) {
    const int64_t cs = c * kEmbChunk, ce = cs + kEmbChunk < n ? cs + kEmbChunk : n;
    for (int64_t j = cs; j < ce;) {
      const int64_t id = sid[j];
      int64_t e = j + 1;
      while (e < ce && sid[e] == id) ++e;
      if (id >= 0 && id < V) {
        const bool cont_in = j == cs && cs > 0 && sid[cs - 1] == id;
        const bool cont_out = e == ce && ce < n && sid[ce] == id;
        float* dst = cont_in ? head + c * d : cont_out ? tail + c * d : gW + id * d;
        for (int col = lane * 4; col < d; col += 256) {
          float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
          for (int64_t k = j; k < e; ++k) {
            const float4 v = get4(dy, perm[k] * d + col);
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
          }
          float4* g = reinterpret_cast<float4*>(dst + col);
          if (!cont_in && !cont_out) {
            const float4 o = *g;
            acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
          }
          *g = acc;
        }
      }
      j = e;
    }
  }
}

__global__ void __launch_bounds__(256) embed_bwd_sorted_join_kernel(const int64_t* __restrict__ sid,
                                                                    float* __restrict__ gW,
                                                                    const float* __restrict__ head,
                                                                    const float* __restrict__ tail, int64_t n, int d,
                                                                    int V) {
  const int lane = threadIdx.x & 63;
  const int64_t nchunks = (n + kEmbChunk - 1) / kEmbChunk;
  for (int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < nchunks; c += (int64_t)gridDim.x * 4) {
    const int64_t cs = c * kEmbChunk, ce = cs + kEmbChunk < n ? cs + kEmbChunk : n;
    const int64_t id = sid[ce - 1];
    if (ce >= n || sid[ce] != id || id < 0 || id >= V) continue;   // last run ends in this chunk
    if (sid[cs] == id && cs > 0 && sid[cs - 1] == id) continue;    // ... or started before it
    for (int col = lane * 4; col < d; col += 256) {
      float4 acc = *reinterpret_cast<const float4*>(tail + c * d + col);
      for (int64_t k = c + 1; k < nchunks; ++k) {
        const float4 v = *reinterpret_cast<const float4*>(head + k * d + col);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        const int64_t ke = (k + 1) * kEmbChunk;
        if (ke >= n || sid[ke] != id) break;
      }
      float4* g = reinterpret_cast<float4*>(gW + id * d + col);
      const float4 o = *g;
      acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
      *g = acc;
    }
  }
}

// ws: 2 * ceil(n / 64) * d floats (head and tail partials); no initialisation needed.
// ddt: dtype of dy (F32 / BF16)
ND_API int nd_embedding_bwd_sorted(const int64_t* sid, const int64_t* perm, const void* dy, int ddt, float* gW,
                                   float* ws, int64_t n, int d, int V, hipStream_t s) {
  if (d % 4) return (int)hipErrorInvalidValue;
  if (n <= 0) return 0;
  const int64_t nchunks = (n + kEmbChunk - 1) / kEmbChunk;
  float* head = ws;
  float* tail = ws + nchunks * d;
  int64_t blocks = (nchunks + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  if (ddt == F32)
    hipLaunchKernelGGL(embed_bwd_sorted_chunks_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s, sid, perm,
                       (const float*)dy, gW, head, tail, n, d, V);
  else if (ddt == BF16)
    hipLaunchKernelGGL(embed_bwd_sorted_chunks_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, s, sid, perm,
                       (const bf16_t*)dy, gW, head, tail, n, d, V);
  else
    return (int)hipErrorInvalidValue;
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(embed_bwd_sorted_join_kernel, dim3((unsigned)blocks), dim3(256), 0, s, sid, gW, head, tail, n, d,
                     V);
  ND_LAUNCH_CHECK();
}

// odt: dtype of out (F32 / BF16)
ND_API int nd_embedding_fwd(const int64_t* ids, const float* W, void* out, int odt, int64_t n, int d, int V,
                            hipStream_t s) {
  if (d % 4) return (int)hipErrorInvalidValue;
  int64_t blocks = (n + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  if (odt == F32)
    hipLaunchKernelGGL(embed_fwd_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s, ids, W, (float*)out, n, d, V);
  else if (odt == BF16)
    hipLaunchKernelGGL(embed_fwd_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, s, ids, W, (bf16_t*)out, n, d,
                       V);
  else
    return (int)hipErrorInvalidValue;
  ND_LAUNCH_CHECK();
}

ND_API int nd_embedding_bwd(const int64_t* ids, const void* dy, int ddt, float* gW, int64_t n, int d, int V,
                            hipStream_t s) {
  int64_t blocks = (n + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  if (ddt == F32)
    hipLaunchKernelGGL(embed_bwd_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s, ids, (const float*)dy, gW, n,
                       d, V);
  else if (ddt == BF16)
    hipLaunchKernelGGL(embed_bwd_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, s, ids, (const bf16_t*)dy, gW,
                       n, d, V);
  else
    return (int)hipErrorInvalidValue;
  ND_LAUNCH_CHECK();
}
