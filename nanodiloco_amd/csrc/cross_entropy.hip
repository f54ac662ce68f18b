// Cross-entropy forward+backward on one chunk of lm_head logits, in place (K9).
//
// One 256-thread workgroup per token row.  For V <= 256*8*CH the whole row is held in registers
// (16-B loads, CH chunks of 8 per thread: V=32000 -> 16 chunks = 64 VGPRs of packed bf16), so the
// row is read from HBM exactly once and written once:
//   m = max(x), s = sum exp(x - m), lse = m + log s            (fp32, block reductions)
//   loss_row = lse - x[target]            -> block sum -> one atomicAdd into loss_sum (or, with
//                                           row_loss != nullptr, one store per row: deterministic)
//   x <- (exp(x - lse) - [j == target]) * scale               (dlogits, compute dtype)
// scale = loss_scale / n_valid lives in device memory (no host sync).  Rows whose target is
// ignore_index contribute 0 loss and 0 gradient.  Larger vocabularies use the two-pass variant.
#include "common.h"
#include <cstdlib>

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
                                                     int V, int ignore, float* __restrict__ lse_out,
                                                     float* __restrict__ row_loss) {
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
  if (threadIdx.x == 0) {
    if (row_loss) row_loss[row] = valid ? lse - picked : 0.f;  // deterministic mode: summed in order later
    else if (valid) atomicAdd(loss_sum, lse - picked);
  }
}


// bf16 rows, packed: the row stays in registers as raw bf16 pairs (CH x 4 VGPRs instead of CH x 8
// fp32), so more waves fit per SIMD to keep the 64-KiB row loads in flight; scores are handled in
// the log2 domain (one FMA + v_exp_f32 per element and pass); the target column is fixed up once by
// the thread that owns it instead of a compare per element.
// QF >= 0 (fp8 lm head, round 5): the dlogits go out ONLY as fp8 (QF: 0 e4m3, 1 e5m2) into q8.q [rows, V], from
// the bf16-rounded values -- bitwise nd_fp8_cast over the bf16 dlogits, whose 4.2 GB write and re-read per
// 65,536-row chunk this removes; amax partials as the other fused producers (common.h Fp8Out).
template <int CH, int QF = -1>
__global__ void __launch_bounds__(256) ce_bf16_kernel(bf16_t* __restrict__ logits, const int64_t* __restrict__ targets,
                                                      float* __restrict__ loss_sum, const float* __restrict__ scale_p,
                                                      int V, int ignore, float* __restrict__ lse_out,
                                                     float* __restrict__ row_loss, Fp8Out q8) {
  constexpr float L2E = 1.4426950408889634f, LN2 = 0.6931471805599453f;
  __shared__ float red[8];
  const int64_t row = blockIdx.x;
  bf16_t* rp = logits + row * (int64_t)V;
  const int tgt = (int)targets[row];
  const bool valid = tgt != ignore;
  uint4 x[CH];
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 256 + threadIdx.x) * 8;
    if (col < V) {
      x[c] = *reinterpret_cast<const uint4*>(rp + col);
      const uint32_t u[4] = {x[c].x, x[c].y, x[c].z, x[c].w};
#pragma unroll
      for (int j = 0; j < 4; ++j) m = fmaxf(m, fmaxf(lo_bf(u[j]), hi_bf(u[j])));
    }
  }
  m = block_max<256>(m, red);
  const float m2 = m * L2E;
  // opaque to the optimiser: stops it from keeping the unpacked fp32 copies alive across passes
#pragma unroll
  for (int c = 0; c < CH; ++c) asm volatile("" : "+v"(x[c].x), "+v"(x[c].y), "+v"(x[c].z), "+v"(x[c].w));
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 256 + threadIdx.x) * 8;
    if (col < V) {
      const uint32_t u[4] = {x[c].x, x[c].y, x[c].z, x[c].w};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        s += __builtin_amdgcn_exp2f(fmaf(lo_bf(u[j]), L2E, -m2)) + __builtin_amdgcn_exp2f(fmaf(hi_bf(u[j]), L2E, -m2));
    }
  }
  __syncthreads();
  s = block_sum<256>(s, red);
  const float lse2 = m2 + __log2f(s);  // log2-domain logsumexp
#pragma unroll
  for (int c = 0; c < CH; ++c) asm volatile("" : "+v"(x[c].x), "+v"(x[c].y), "+v"(x[c].z), "+v"(x[c].w));
  const float sc = valid ? scale_p[0] : 0.f;
  const float qsc = QF >= 0 ? q8.scale[0] : 1.f;
  float qmax = 0.f;
  float picked = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int col = (c * 256 + threadIdx.x) * 8;
    if (col < V) {
      const uint32_t u[4] = {x[c].x, x[c].y, x[c].z, x[c].w};
      float o[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[2 * j] = __builtin_amdgcn_exp2f(fmaf(lo_bf(u[j]), L2E, -lse2)) * sc;
        o[2 * j + 1] = __builtin_amdgcn_exp2f(fmaf(hi_bf(u[j]), L2E, -lse2)) * sc;
      }
      const unsigned d = (unsigned)(tgt - col);
      if (d < 8u) {  // this thread owns the target column
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if ((unsigned)j == d) {
            picked = (j & 1) ? hi_bf(u[j >> 1]) : lo_bf(u[j >> 1]);
            o[j] -= sc;
          }
      }
      uint4 w;
      w.x = pack2(o[0], o[1]); w.y = pack2(o[2], o[3]); w.z = pack2(o[4], o[5]); w.w = pack2(o[6], o[7]);
      if constexpr (QF < 0) {
        *reinterpret_cast<uint4*>(rp + col) = w;
      } else {
        const float r[8] = {lo_bf(w.x), hi_bf(w.x), lo_bf(w.y), hi_bf(w.y), lo_bf(w.z), hi_bf(w.z), lo_bf(w.w), hi_bf(w.w)};
#pragma unroll
        for (int j = 0; j < 8; ++j) qmax = fmaxf(qmax, fabsf(r[j]));
        uint2 o8;
        o8.x = cvt4<QF>(r[0] * qsc, r[1] * qsc, r[2] * qsc, r[3] * qsc);
        o8.y = cvt4<QF>(r[4] * qsc, r[5] * qsc, r[6] * qsc, r[7] * qsc);
        *reinterpret_cast<uint2*>(q8.q + row * (int64_t)V + col) = o8;
      }
    }
  }
  if constexpr (QF >= 0) block_amax_commit<256>(qmax, q8.amax, q8.parts);
  const float lse = lse2 * LN2;
  if (threadIdx.x == 0 && lse_out) lse_out[row] = lse;
  __syncthreads();
  picked = block_sum<256>(picked, red);
  if (threadIdx.x == 0) {
    if (row_loss) row_loss[row] = valid ? lse - picked : 0.f;  // deterministic mode: summed in order later
    else if (valid) atomicAdd(loss_sum, lse - picked);
  }
}

// Generic two-pass variant (any V, scalar accesses): online max/sum, then gradient write.
template <int DT>
__global__ void __launch_bounds__(256) ce_generic_kernel(void* __restrict__ logits, const int64_t* __restrict__ targets,
                                                         float* __restrict__ loss_sum, const float* __restrict__ scale_p,
                                                         int V, int ignore, float* __restrict__ lse_out,
                                                     float* __restrict__ row_loss) {
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
  if (threadIdx.x == 0) {
    if (row_loss) row_loss[row] = valid ? lse - picked : 0.f;  // deterministic mode: summed in order later
    else if (valid) atomicAdd(loss_sum, lse - picked);
  }
}

// ND_CE=r: the register kernel for bf16 rows too (A/B), read once at load
static const bool g_ce_reg = [] {
  const char* e = getenv("ND_CE");
  return e && e[0] == 'r';
}();

ND_API int nd_ce_fwd_bwd(void* logits, int dt, const int64_t* targets, float* loss_sum, const float* scale,
                         int64_t n, int V, int ignore, float* lse_out, float* row_loss, float /*reserved*/,
                         hipStream_t s) {
  if (n <= 0) return 0;
  dim3 g((unsigned)n), b(256);
  if (V % 8 == 0 && V <= 256 * 8 * 16) {
    if (V <= 256 * 8 * 4) {
      if (dt == BF16) hipLaunchKernelGGL((ce_reg_kernel<BF16, 4>), g, b, 0, s, logits, targets, loss_sum, scale, V, ignore, lse_out, row_loss);
      else hipLaunchKernelGGL((ce_reg_kernel<F32, 4>), g, b, 0, s, logits, targets, loss_sum, scale, V, ignore, lse_out, row_loss);
    } else {
      if (dt == BF16 && !g_ce_reg)
        hipLaunchKernelGGL((ce_bf16_kernel<16>), g, b, 0, s, (bf16_t*)logits, targets, loss_sum, scale, V, ignore, lse_out, row_loss,
                           Fp8Out{nullptr, nullptr, nullptr, 1, 0});
      else if (dt == BF16) hipLaunchKernelGGL((ce_reg_kernel<BF16, 16>), g, b, 0, s, logits, targets, loss_sum, scale, V, ignore, lse_out, row_loss);
      else hipLaunchKernelGGL((ce_reg_kernel<F32, 16>), g, b, 0, s, logits, targets, loss_sum, scale, V, ignore, lse_out, row_loss);
    }
  } else {
    if (dt == BF16) hipLaunchKernelGGL(ce_generic_kernel<BF16>, g, b, 0, s, logits, targets, loss_sum, scale, V, ignore, lse_out, row_loss);
    else hipLaunchKernelGGL(ce_generic_kernel<F32>, g, b, 0, s, logits, targets, loss_sum, scale, V, ignore, lse_out, row_loss);
  }
  ND_LAUNCH_CHECK();
}

// fp8 lm head: the same loss / gradient with the dlogits written only as fp8 (q: [n, V] bytes; e4m3 or e5m2 by fmt,
// qscale = device scalar, amax = `parts` partial maxima).  Only the packed bf16 kernel's shapes (V % 8 == 0,
// 8192 < V <= 32768, bf16 logits); anything else returns hipErrorInvalidValue and the caller casts separately.
// The logits buffer is left as the forward wrote it.
ND_API int nd_ce_fwd_bwd_q8(void* logits, int dt, const int64_t* targets, float* loss_sum, const float* scale,
                            int64_t n, int V, int ignore, float* lse_out, float* row_loss, void* q, const float* qscale,
                            float* amax, int parts, int fmt, hipStream_t s) {
  if (n <= 0) return 0;
  if (dt != BF16 || V % 8 != 0 || V <= 256 * 8 * 4 || V > 256 * 8 * 16 || g_ce_reg || !q || !qscale || !amax ||
      parts < 1 || (fmt != 0 && fmt != 1))
    return (int)hipErrorInvalidValue;
  const Fp8Out q8{(uint8_t*)q, qscale, amax, parts, fmt};
  dim3 g((unsigned)n), b(256);
  if (fmt == 0)
    hipLaunchKernelGGL((ce_bf16_kernel<16, 0>), g, b, 0, s, (bf16_t*)logits, targets, loss_sum, scale, V, ignore, lse_out,
                       row_loss, q8);
  else
    hipLaunchKernelGGL((ce_bf16_kernel<16, 1>), g, b, 0, s, (bf16_t*)logits, targets, loss_sum, scale, V, ignore, lse_out,
                       row_loss, q8);
  ND_LAUNCH_CHECK();
}
