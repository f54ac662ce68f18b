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

__global__ void __launch_bounds__(256) embed_bwd_sorted_chunks_kernel(const int64_t* __restrict__ sid,
                                                                      const int64_t* __restrict__ perm,
                                                                      const float* __restrict__ dy,
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
            const float4 v = *reinterpret_cast<const float4*>(dy + perm[k] * d + col);
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
ND_API int nd_embedding_bwd_sorted(const int64_t* sid, const int64_t* perm, const float* dy, float* gW, float* ws,
                                   int64_t n, int d, int V, hipStream_t s) {
  if (d % 4) return (int)hipErrorInvalidValue;
  if (n <= 0) return 0;
  const int64_t nchunks = (n + kEmbChunk - 1) / kEmbChunk;
  float* head = ws;
  float* tail = ws + nchunks * d;
  int64_t blocks = (nchunks + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(embed_bwd_sorted_chunks_kernel, dim3((unsigned)blocks), dim3(256), 0, s, sid, perm, dy, gW, head,
                     tail, n, d, V);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(embed_bwd_sorted_join_kernel, dim3((unsigned)blocks), dim3(256), 0, s, sid, gW, head, tail, n, d,
                     V);
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
