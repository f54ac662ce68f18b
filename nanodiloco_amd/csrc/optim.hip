// Flat-buffer optimizer kernels (K12-K17): grad-norm partials, fused clip+AdamW with bf16 shadow
// write-out, DiLoCo pseudo-gradient, fused outer SGD-Nesterov.
//
// All are pure HBM streams over 16-B vectors with grid-stride loops (grid capped at 2048 blocks,
// Guideline 11).  The clip coefficient never touches the host: nd_adamw_step re-reduces the
// <=1024 per-block sum-of-squares partials in every block (4 KB, L2-resident) before its stream.
#include "common.h"

using namespace nd;

static unsigned stream_grid(int64_t n4) {
  int64_t b = (n4 + 255) / 256;
  return (unsigned)(b > 2048 ? 2048 : (b < 1 ? 1 : b));
}

__global__ void __launch_bounds__(256) sumsq_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ part) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t n4 = n >> 2;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 v = g4[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    acc += g[i] * g[i];
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

ND_API int nd_sumsq_partial(const float* g, int64_t n, float* part, int nblocks, hipStream_t s) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblocks), dim3(256), 0, s, g, n, part);
  ND_LAUNCH_CHECK();
}

template <int SDT>
__global__ void __launch_bounds__(256) adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, void* __restrict__ sh,
                                                    int64_t n, const float* __restrict__ part, int nparts, float lr,
                                                    float b1, float b2, float eps, float wd, float bc1, float bc2,
                                                    float max_norm, float* __restrict__ norm_out, int skip_nonfinite,
                                                    int* __restrict__ skipped) {
  __shared__ float red[4];
  float coef = 1.f;
  if (part) {
    float t = 0.f;
    for (int i = threadIdx.x; i < nparts; i += 256) t += part[i];
    t = block_sum<256>(t, red);
    const float norm = sqrtf(t);
    if (max_norm > 0.f) coef = fminf(1.f, max_norm / (norm + 1e-6f));
    if (norm_out && blockIdx.x == 0 && threadIdx.x == 0) norm_out[0] = norm;
    // device-side guard: every block sees the same norm, so a NaN/Inf step is skipped everywhere
    // (no host sync); the step counter on the host still advances, like torch's GradScaler skip.
    if (skip_nonfinite && !isfinite(norm)) {
      if (skipped && blockIdx.x == 0 && threadIdx.x == 0) skipped[0] += 1;
      return;
    }
  }
  const float decay = 1.f - lr * wd;
  const float step = lr / bc1;
  const float rbc2 = 1.f / sqrtf(bc2);
  const float omb1 = 1.f - b1, omb2 = 1.f - b2;
  auto upd = [&](float& pp, float gg, float& mm, float& vv) {
    gg *= coef;
    pp *= decay;
    mm = mm + omb1 * (gg - mm);
    vv = vv * b2 + omb2 * gg * gg;
    const float den = sqrtf(vv) * rbc2 + eps;
    pp = pp - step * (mm / den);
  };
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 P = reinterpret_cast<float4*>(p)[i];
    const float4 G = reinterpret_cast<const float4*>(g)[i];
    float4 M = reinterpret_cast<float4*>(m)[i];
    float4 Vv = reinterpret_cast<float4*>(v)[i];
    upd(P.x, G.x, M.x, Vv.x);
    upd(P.y, G.y, M.y, Vv.y);
    upd(P.z, G.z, M.z, Vv.z);
    upd(P.w, G.w, M.w, Vv.w);
    reinterpret_cast<float4*>(p)[i] = P;
    reinterpret_cast<float4*>(m)[i] = M;
    reinterpret_cast<float4*>(v)[i] = Vv;
    if (SDT == BF16)
      reinterpret_cast<uint2*>(sh)[i] = make_uint2(pack2(P.x, P.y), pack2(P.z, P.w));
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float pp = p[i], mm = m[i], vv = v[i];
    upd(pp, g[i], mm, vv);
    p[i] = pp; m[i] = mm; v[i] = vv;
    if (SDT == BF16) reinterpret_cast<bf16_t*>(sh)[i] = f2bf(pp);
  }
}

ND_API int nd_adamw_step(float* p, const float* g, float* m, float* v, void* sh, int shdt, int64_t n,
                         const float* part, int nparts, float lr, float b1, float b2, float eps, float wd, float bc1,
                         float bc2, float max_norm, float* norm_out, int skip_nonfinite, int* skipped, hipStream_t s) {
  const unsigned grid = stream_grid(n >> 2);
  if (sh && shdt == BF16)
    hipLaunchKernelGGL(adamw_kernel<BF16>, dim3(grid), dim3(256), 0, s, p, g, m, v, sh, n, part, nparts, lr, b1, b2, eps,
                       wd, bc1, bc2, max_norm, norm_out, skip_nonfinite, skipped);
  else
    hipLaunchKernelGGL(adamw_kernel<F32>, dim3(grid), dim3(256), 0, s, p, g, m, v, nullptr, n, part, nparts, lr, b1, b2,
                       eps, wd, bc1, bc2, max_norm, norm_out, skip_nonfinite, skipped);
  ND_LAUNCH_CHECK();
}

template <int DDT>
__global__ void __launch_bounds__(256) pseudograd_kernel(const float* __restrict__ sync, const float* __restrict__ p,
                                                         void* __restrict__ d, int64_t n) {
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 S = reinterpret_cast<const float4*>(sync)[i];
    const float4 P = reinterpret_cast<const float4*>(p)[i];
    const float4 D = make_float4(S.x - P.x, S.y - P.y, S.z - P.z, S.w - P.w);
    if (DDT == BF16) reinterpret_cast<uint2*>(d)[i] = make_uint2(pack2(D.x, D.y), pack2(D.z, D.w));
    else reinterpret_cast<float4*>(d)[i] = D;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float D = sync[i] - p[i];
    if (DDT == BF16) reinterpret_cast<bf16_t*>(d)[i] = f2bf(D);
    else reinterpret_cast<float*>(d)[i] = D;
  }
}

ND_API int nd_pseudograd(const float* sync, const float* p, void* d, int ddt, int64_t n, hipStream_t s) {
  const unsigned grid = stream_grid(n >> 2);
  if (ddt == BF16) hipLaunchKernelGGL(pseudograd_kernel<BF16>, dim3(grid), dim3(256), 0, s, sync, p, d, n);
  else hipLaunchKernelGGL(pseudograd_kernel<F32>, dim3(grid), dim3(256), 0, s, sync, p, d, n);
  ND_LAUNCH_CHECK();
}

// buf = first ? d : mu*buf + d ;  theta = sync - lr*(d + mu*buf) ;  d = delta_sum * inv_world
// drift (optional): p = theta + (p - (sync_old - drift_base)); else p = theta.  sync = theta.
template <int DDT, int SDT>
__global__ void __launch_bounds__(256) outer_kernel(float* __restrict__ p, float* __restrict__ sync,
                                                    const void* __restrict__ dsum, float* __restrict__ buf,
                                                    void* __restrict__ sh, int64_t n, float inv_w, float lr, float mu,
                                                    int first, const float* __restrict__ drift) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float d = (DDT == BF16 ? bf2f(reinterpret_cast<const bf16_t*>(dsum)[i]) : reinterpret_cast<const float*>(dsum)[i]) * inv_w;
    const float b = first ? d : mu * buf[i] + d;
    buf[i] = b;
    const float so = sync[i];
    const float th = so - lr * (d + mu * b);
    const float np = drift ? th + (p[i] - (so - drift[i])) : th;
    sync[i] = th;
    p[i] = np;
    if (SDT == BF16) reinterpret_cast<bf16_t*>(sh)[i] = f2bf(np);
  }
}

ND_API int nd_outer_nesterov(float* p, float* sync, const void* dsum, int ddt, float* buf, void* sh, int shdt, int64_t n,
                             float inv_w, float lr, float mu, int first, const float* drift, void* /*reserved*/,
                             hipStream_t s) {
  int64_t b = (n + 255) / 256;
  const unsigned grid = (unsigned)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
  const bool bsh = sh && shdt == BF16;
#define ND_OK(D, S) hipLaunchKernelGGL((outer_kernel<D, S>), dim3(grid), dim3(256), 0, s, p, sync, dsum, buf, sh, n, inv_w, lr, mu, first, drift)
  if (ddt == BF16) { if (bsh) ND_OK(BF16, BF16); else ND_OK(BF16, F32); }
  else { if (bsh) ND_OK(F32, BF16); else ND_OK(F32, F32); }
#undef ND_OK
  ND_LAUNCH_CHECK();
}

__global__ void axpby_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n, float a, float b) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) y[i] = a * x[i] + b * y[i];
}

ND_API int nd_axpby(const float* x, float* y, int64_t n, float a, float b, hipStream_t s) {
  hipLaunchKernelGGL(axpby_kernel, dim3(stream_grid(n)), dim3(256), 0, s, x, y, n, a, b);
  ND_LAUNCH_CHECK();
}

ND_API int nd_version() { return 1; }
