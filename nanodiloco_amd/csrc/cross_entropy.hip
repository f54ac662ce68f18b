// Cross-entropy forward+backward on one chunk of lm_head logits, in place (K9).
//
// One 256-thread workgroup per token row.  For V <= 256*8*CH the whole row is held in registers
// (16-B loads, CH chunks of 8 per thread: V=32000 -> 16 chunks = 64 VGPRs of packed bf16), so the
// row is read from HBM exactly once and written once:
//   m = max(x), s = sum exp(x - m), lse = m + log s            (fp32, block reductions)
//   loss_row = lse - x[target]            -> block sum -> one atomicAdd into loss_sum
//   x <- (exp(x - lse) - [j == target]) * scale               (dlogits, compute dtype)
// scale = loss_scale / n_valid lives in device memory (no host sync).  Rows whose target is
// ignore_index contribute 0 loss and 0 gradient.  Larger vocabularies use the two-pass variant.
#include "common.h"

using namespace nd;

template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = red[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) t = fmaxf(t, red[i]);
  return t;
}

template <int DT, int CH>
__global__ void __launch_bounds__(256) ce_reg_kernel(void* __restrict__ logits, const int64_t* __restrict__ targets,
                                                     float* __restrict__ loss_sum, const float* __restrict__ scale_p,
                                                     int V, int ignore, float* __restrict__ lse_out) {
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  const int64_t base = row * (int64_t)V;
  const int64_t tgt = targets[row];
  const bool valid = tgt != ignore;
  float x[CH][8];
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 256 + threadIdx.x) * 8;
    if (col < V) {
      Vec8<DT>::load(logits, base + col, x[c]);
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, x[c][j]);
    }
  }
  m = block_max<256>(m, red);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 256 + threadIdx.x) * 8;
    if (col < V) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(x[c][j] - m);
    }
  }
  __syncthreads();
  s = block_sum<256>(s, red);
  const float lse = m + __logf(s);
  const float sc = valid ? scale_p[0] : 0.f;
  float picked = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 256 + threadIdx.x) * 8;
    if (col < V) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool hit = (int64_t)(col + j) == tgt;
        if (hit) picked = x[c][j];
        o[j] = (__expf(x[c][j] - lse) - (hit ? 1.f : 0.f)) * sc;
      }
      Vec8<DT>::store(logits, base + col, o);
    }
  }
  if (threadIdx.x == 0) {
    if (lse_out) lse_out[row] = lse;
  }
  __syncthreads();
  picked = block_sum<256>(picked, red);
  if (threadIdx.x == 0 && valid) atomicAdd(loss_sum, lse - picked);
}

// Generic two-pass variant (any V, scalar accesses): online max/sum, then gradient write.
template <int DT>
__global__ void __launch_bounds__(256) ce_generic_kernel(void* __restrict__ logits, const int64_t* __restrict__ targets,
                                                         float* __restrict__ loss_sum, const float* __restrict__ scale_p,
                                                         int V, int ignore, float* __restrict__ lse_out) {
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  const int64_t base = row * (int64_t)V;
  const int64_t tgt = targets[row];
  const bool valid = tgt != ignore;
  auto ld = [&](int j) -> float {
    if (DT == BF16) return bf2f(reinterpret_cast<const bf16_t*>(logits)[base + j]);
    return reinterpret_cast<const float*>(logits)[base + j];
  };
  float m = -INFINITY, s = 0.f;
  for (int j = threadIdx.x; j < V; j += 256) {
    const float v = ld(j);
    const float nm = fmaxf(m, v);
    s = s * __expf(m - nm) + __expf(v - nm);
    m = nm;
  }
  const float gm = block_max<256>(m, red);
  s = s * __expf(m - gm);
  __syncthreads();
  s = block_sum<256>(s, red);
  const float lse = gm + __logf(s);
  const float sc = valid ? scale_p[0] : 0.f;
  float picked = 0.f;
  for (int j = threadIdx.x; j < V; j += 256) {
    const float v = ld(j);
    const bool hit = (int64_t)j == tgt;
    if (hit) picked = v;
    const float o = (__expf(v - lse) - (hit ? 1.f : 0.f)) * sc;
    if (DT == BF16) reinterpret_cast<bf16_t*>(logits)[base + j] = f2bf(o);
    else reinterpret_cast<float*>(logits)[base + j] = o;
  }
  if (threadIdx.x == 0 && lse_out) lse_out[row] = lse;
  __syncthreads();
  picked = block_sum<256>(picked, red);
  if (threadIdx.x == 0 && valid) atomicAdd(loss_sum, lse - picked);
}

ND_API int nd_ce_fwd_bwd(void* logits, int dt, const int64_t* targets, float* loss_sum, const float* scale,
                         int64_t n, int V, int ignore, float* lse_out, void* /*reserved*/, float /*reserved*/,
                         hipStream_t s) {
  if (n <= 0) return 0;
  dim3 g((unsigned)n), b(256);
  if (V % 8 == 0 && V <= 256 * 8 * 16) {
    if (V <= 256 * 8 * 4) {
      if (dt == BF16) hipLaunchKernelGGL((ce_reg_kernel<BF16, 4>), g, b, 0, s, logits, targets, loss_sum, scale, V, ignore, lse_out);
      else hipLaunchKernelGGL((ce_reg_kernel<F32, 4>), g, b, 0, s, logits, targets, loss_sum, scale, V, ignore, lse_out);
    } else {
      if (dt == BF16) hipLaunchKernelGGL((ce_reg_kernel<BF16, 16>), g, b, 0, s, logits, targets, loss_sum, scale, V, ignore, lse_out);
      else hipLaunchKernelGGL((ce_reg_kernel<F32, 16>), g, b, 0, s, logits, targets, loss_sum, scale, V, ignore, lse_out);
    }
  } else {
    if (dt == BF16) hipLaunchKernelGGL(ce_generic_kernel<BF16>, g, b, 0, s, logits, targets, loss_sum, scale, V, ignore, lse_out);
    else hipLaunchKernelGGL(ce_generic_kernel<F32>, g, b, 0, s, logits, targets, loss_sum, scale, V, ignore, lse_out);
  }
  ND_LAUNCH_CHECK();
}
