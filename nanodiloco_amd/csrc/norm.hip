// RMSNorm (+ fused residual add) forward / backward for gfx950.
//
// Memory-bound: one 64-lane wave owns one row; each lane holds NCH chunks of 8 contiguous
// elements (16-B bf16 / 32-B fp32 vector accesses, Guideline 13), so a row is read exactly once
// from HBM and reduced with a wave butterfly (no LDS, no block barrier in the forward).
// Forward fuses h_new = h + a (residual, fp32) with y = w * h_new * rstd (compute dtype) and
// saves rstd.  Backward recomputes xhat from (h_new, rstd), adds the incoming residual gradient,
// emits dx (fp32) and optionally the branch gradient in the compute dtype, and accumulates
// dw = sum_rows dy * xhat per lane in registers across the rows a wave visits; the 4 waves of a
// block combine through LDS and write one partial row per block (host reduces <=1024 partials).
// Residual stream dtype (round 5): fp32 by default; bf16 (`--residual-dtype bf16`, Megatron's default) keeps
// h_new, the incoming residual gradient and dx in bf16 -- h_new is rounded BEFORE the statistics so the
// backward's recomputed xhat matches, and dx doubles as the branch gradient (one bf16 store instead of an fp32
// dx plus a bf16 da): the forward moves 4 instead of 6 bf16-tensor units, the backward 4 instead of 8.
#include "common.h"

using namespace nd;

// Q (YDT == BF16 only): fused fp8 side output of y for the fp8 inner step (common.h Fp8Out).
template <int NCH, int XDT, int ADT, int YDT, bool Q = false>
__global__ void __launch_bounds__(256) rmsnorm_fwd_kernel(const void* __restrict__ x, const void* __restrict__ a,
                                                          const float* __restrict__ w, void* __restrict__ y,
                                                          void* __restrict__ h_out, float* __restrict__ rstd_out,
                                                          int64_t rows, int cols, float eps, Fp8Out q8) {
  float qmax = 0.f;
  const float qsc = Q ? q8.scale[0] : 1.f;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t r = wave; r < rows; r += nwaves) {
    float v[NCH][8];
    float ss = 0.f;
    const int64_t base = r * cols;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (col < cols) {
        Vec8<XDT>::load(x, base + col, v[c]);
        if (ADT >= 0) {
          float t[8];
          Vec8<(ADT >= 0 ? ADT : 0)>::load(a, base + col, t);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[c][j] += t[j];
          if (XDT == BF16) round_bf16x8(v[c]);  // bf16 residual: statistics of the stored h_new
          Vec8<XDT>::store(h_out, base + col, v[c]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
      }
    }
    ss = wave_sum(ss);
    const float rs = rsqrtf(ss / (float)cols + eps);
    if (lane == 0) rstd_out[r] = rs;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (col < cols) {
        float wv[8], o[8];
        Vec8<F32>::load(w, col, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = wv[j] * (v[c][j] * rs);
        if (Q) put8_bf16_q(y, base + col, o, q8, qsc, qmax);  // YDT == BF16 (launcher)
        else Vec8<YDT>::store(y, base + col, o);
      }
    }
  }
  if (Q) block_amax_commit<256>(qmax, q8.amax, q8.parts);
}

// Q (DADT == BF16 only): fused fp8 side output of the branch gradient da (common.h Fp8Out).
// HDT: residual dtype of h, dres and dx.  HDT == BF16 with a bf16 branch gradient: da IS dx (host passes the
// same pointer) and only the da store runs.
template <int NCH, int DYDT, int DADT, bool Q = false, int HDT = F32>
__global__ void __launch_bounds__(256, (NCH <= 2 ? 4 : 1)) rmsnorm_bwd_kernel(const void* __restrict__ dy, const void* __restrict__ h,
                                                          const float* __restrict__ w, const float* __restrict__ rstd,
                                                          const void* __restrict__ dres, void* dx,
                                                          void* da, float* __restrict__ part,
                                                          int64_t rows, int cols, Fp8Out q8) {
  constexpr bool DXA = HDT == BF16 && (Q || DADT == BF16);  // dx aliases da
  float qmax = 0.f;
  const float qsc = Q ? q8.scale[0] : 1.f;
  extern __shared__ __attribute__((aligned(16))) float sdw[];  // [4 waves][cols] weight-gradient partials
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  float dwacc[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[c][j] = 0.f;
  float wv[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < cols) Vec8<F32>::load(w, col, wv[c]);
  }
  for (int64_t r = wave; r < rows; r += nwaves) {
    const int64_t base = r * cols;
    const float rs = rstd[r];
    float g[NCH][8], xh[NCH][8];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (col < cols) {
        float d[8];
        Vec8<DYDT>::load(dy, base + col, d);
        Vec8<HDT>::load(h, base + col, xh[c]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[c][j] *= rs;
          g[c][j] = d[j] * wv[c][j];
          dot += g[c][j] * xh[c][j];
          dwacc[c][j] += d[j] * xh[c][j];
        }
      }
    }
    dot = wave_sum(dot) / (float)cols;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (col < cols) {
        float o[8];
        if (dres) Vec8<HDT>::load(dres, base + col, o);
        else {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += rs * (g[c][j] - xh[c][j] * dot);
        if (!DXA) Vec8<HDT>::store(dx, base + col, o);
        if (Q) put8_bf16_q(da, base + col, o, q8, qsc, qmax);  // DADT == BF16 (launcher)
        else if (DADT >= 0) Vec8<(DADT >= 0 ? DADT : 0)>::store(da, base + col, o);
      }
    }
  }
  if (Q) block_amax_commit<256>(qmax, q8.amax, q8.parts);
  // each wave stores its partial row; the block's four are summed in wave order (no LDS float
  // atomics: their arrival order made the weight gradient non-reproducible in the last bits)
  float* mine = sdw + (threadIdx.x >> 6) * cols;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < cols) Vec8<F32>::store(mine, col, dwacc[c]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < cols; i += 256)
    part[(int64_t)blockIdx.x * cols + i] = ((sdw[i] + sdw[cols + i]) + sdw[2 * cols + i]) + sdw[3 * cols + i];
}

// ------------------------------------------------------------------------------------ launchers
template <int NCH>
static int fwd_dispatch(const void* x, int xdt, const void* a, int adt, const float* w, void* y, int ydt, void* h,
                        float* rstd, int64_t rows, int cols, float eps, hipStream_t s, const Fp8Out* q8 = nullptr) {
  int64_t blocks = (rows + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  dim3 g((unsigned)blocks), b(256);
  const Fp8Out none{nullptr, nullptr, nullptr, 1, 0};
  if (q8) {  // fused fp8 side output: bf16 y only
    if (ydt != BF16 || (xdt != F32 && xdt != BF16) || (a != nullptr && adt != BF16)) return (int)hipErrorInvalidValue;
    if (a == nullptr && xdt == F32)
      hipLaunchKernelGGL((rmsnorm_fwd_kernel<NCH, F32, -1, BF16, true>), g, b, 0, s, x, a, w, y, h, rstd, rows, cols,
                         eps, *q8);
    else if (a == nullptr)
      hipLaunchKernelGGL((rmsnorm_fwd_kernel<NCH, BF16, -1, BF16, true>), g, b, 0, s, x, a, w, y, h, rstd, rows, cols,
                         eps, *q8);
    else if (xdt == F32)
      hipLaunchKernelGGL((rmsnorm_fwd_kernel<NCH, F32, BF16, BF16, true>), g, b, 0, s, x, a, w, y, h, rstd, rows, cols,
                         eps, *q8);
    else
      hipLaunchKernelGGL((rmsnorm_fwd_kernel<NCH, BF16, BF16, BF16, true>), g, b, 0, s, x, a, w, y, h, rstd, rows, cols,
                         eps, *q8);
    ND_LAUNCH_CHECK();
  }
#define ND_RF(X, A, Y) hipLaunchKernelGGL((rmsnorm_fwd_kernel<NCH, X, A, Y>), g, b, 0, s, x, a, w, y, h, rstd, rows, cols, eps, none)
  if (a == nullptr) {
    if (xdt == F32 && ydt == BF16) ND_RF(F32, -1, BF16);
    else if (xdt == F32 && ydt == F32) ND_RF(F32, -1, F32);
    else if (xdt == BF16 && ydt == BF16) ND_RF(BF16, -1, BF16);
    else return (int)hipErrorInvalidValue;
  } else {
    if (xdt == F32 && adt == BF16 && ydt == BF16) ND_RF(F32, BF16, BF16);
    else if (xdt == F32 && adt == F32 && ydt == F32) ND_RF(F32, F32, F32);
    else if (xdt == F32 && adt == F32 && ydt == BF16) ND_RF(F32, F32, BF16);
    else if (xdt == BF16 && adt == BF16 && ydt == BF16) ND_RF(BF16, BF16, BF16);
    else return (int)hipErrorInvalidValue;
  }
#undef ND_RF
  ND_LAUNCH_CHECK();
}

ND_API int nd_rmsnorm_fwd(const void* x, int xdt, const void* a, int adt, const float* w, void* y, int ydt, void* h,
                          float* rstd, int64_t rows, int cols, float eps, hipStream_t s) {
  if (cols % 8 || cols > 8 * 512) return (int)hipErrorInvalidValue;
  const int nch = (cols + 511) / 512;
  switch (nch) {
    case 1: return fwd_dispatch<1>(x, xdt, a, adt, w, y, ydt, h, rstd, rows, cols, eps, s);
    case 2: return fwd_dispatch<2>(x, xdt, a, adt, w, y, ydt, h, rstd, rows, cols, eps, s);
    case 3: case 4: return fwd_dispatch<4>(x, xdt, a, adt, w, y, ydt, h, rstd, rows, cols, eps, s);
    default: return fwd_dispatch<8>(x, xdt, a, adt, w, y, ydt, h, rstd, rows, cols, eps, s);
  }
}

template <int NCH>
static int bwd_dispatch(const void* dy, int dydt, const void* h, int hdt, const float* w, const float* rstd,
                        const void* dres, void* dx, int dadt, void* da, int64_t rows, int cols, float* part, hipStream_t s,
                        const Fp8Out* q8 = nullptr) {
  int64_t blocks = (rows + 63) / 64;
  if (blocks > 1024) blocks = 1024;
  dim3 g((unsigned)blocks), b(256);
  size_t lds = 4 * (size_t)cols * sizeof(float);
  const Fp8Out none{nullptr, nullptr, nullptr, 1, 0};
  if (q8) {  // fused fp8 side output: bf16 dy and da only
    if (dydt != BF16 || dadt != BF16 || da == nullptr) return (int)hipErrorInvalidValue;
    if (hdt == F32)
      hipLaunchKernelGGL((rmsnorm_bwd_kernel<NCH, BF16, BF16, true>), g, b, lds, s, dy, h, w, rstd, dres, dx, da, part,
                         rows, cols, *q8);
    else if (hdt == BF16 && da == dx)
      hipLaunchKernelGGL((rmsnorm_bwd_kernel<NCH, BF16, BF16, true, BF16>), g, b, lds, s, dy, h, w, rstd, dres, dx, da,
                         part, rows, cols, *q8);
    else
      return (int)hipErrorInvalidValue;
    ND_LAUNCH_CHECK();
  }
  if (hdt == BF16) {  // bf16 residual: bf16 dy; the branch gradient (if any) is dx itself
    if (dydt != BF16 || (da != nullptr && (dadt != BF16 || da != dx))) return (int)hipErrorInvalidValue;
    if (da == nullptr)
      hipLaunchKernelGGL((rmsnorm_bwd_kernel<NCH, BF16, -1, false, BF16>), g, b, lds, s, dy, h, w, rstd, dres, dx, da,
                         part, rows, cols, none);
    else
      hipLaunchKernelGGL((rmsnorm_bwd_kernel<NCH, BF16, BF16, false, BF16>), g, b, lds, s, dy, h, w, rstd, dres, dx, da,
                         part, rows, cols, none);
    ND_LAUNCH_CHECK();
  }
  if (hdt != F32) return (int)hipErrorInvalidValue;
#define ND_RB(D, A) hipLaunchKernelGGL((rmsnorm_bwd_kernel<NCH, D, A>), g, b, lds, s, dy, h, w, rstd, dres, dx, da, part, rows, cols, none)
  if (da == nullptr) {
    if (dydt == BF16) ND_RB(BF16, -1); else ND_RB(F32, -1);
  } else {
    if (dydt == BF16 && dadt == BF16) ND_RB(BF16, BF16);
    else if (dydt == F32 && dadt == F32) ND_RB(F32, F32);
    else if (dydt == BF16 && dadt == F32) ND_RB(BF16, F32);
    else ND_RB(F32, BF16);
  }
#undef ND_RB
  ND_LAUNCH_CHECK();
}

// part must hold min(1024, ceil(rows/64)) * cols floats (the Python side allocates exactly that).
// hdt: dtype of h, dres and dx (F32, or BF16 with da == dx or da == nullptr)
ND_API int nd_rmsnorm_bwd(const void* dy, int dydt, const void* h, int hdt, const float* w, const float* rstd,
                          const void* dres, void* dx, int dadt, void* da, int64_t rows, int cols, float* part,
                          hipStream_t s) {
  if (cols % 8 || cols > 8 * 512) return (int)hipErrorInvalidValue;
  const int nch = (cols + 511) / 512;
  switch (nch) {
    case 1: return bwd_dispatch<1>(dy, dydt, h, hdt, w, rstd, dres, dx, dadt, da, rows, cols, part, s);
    case 2: return bwd_dispatch<2>(dy, dydt, h, hdt, w, rstd, dres, dx, dadt, da, rows, cols, part, s);
    case 3: case 4: return bwd_dispatch<4>(dy, dydt, h, hdt, w, rstd, dres, dx, dadt, da, rows, cols, part, s);
    default: return bwd_dispatch<8>(dy, dydt, h, hdt, w, rstd, dres, dx, dadt, da, rows, cols, part, s);
  }
}

// fp8 inner step: the same launchers with the fused fp8 side output (q: fp8 bytes shaped like y / da).
ND_API int nd_rmsnorm_fwd_q(const void* x, int xdt, const void* a, int adt, const float* w, void* y, int ydt, void* h,
                            float* rstd, int64_t rows, int cols, float eps, void* q, const float* scale, float* amax,
                            int parts, int fmt, hipStream_t s) {
  if (cols % 8 || cols > 8 * 512 || !q || !scale || !amax || parts < 1) return (int)hipErrorInvalidValue;
  const Fp8Out q8{(uint8_t*)q, scale, amax, parts, fmt};
  switch ((cols + 511) / 512) {
    case 1: return fwd_dispatch<1>(x, xdt, a, adt, w, y, ydt, h, rstd, rows, cols, eps, s, &q8);
    case 2: return fwd_dispatch<2>(x, xdt, a, adt, w, y, ydt, h, rstd, rows, cols, eps, s, &q8);
    case 3: case 4: return fwd_dispatch<4>(x, xdt, a, adt, w, y, ydt, h, rstd, rows, cols, eps, s, &q8);
    default: return fwd_dispatch<8>(x, xdt, a, adt, w, y, ydt, h, rstd, rows, cols, eps, s, &q8);
  }
}

ND_API int nd_rmsnorm_bwd_q(const void* dy, int dydt, const void* h, int hdt, const float* w, const float* rstd,
                            const void* dres, void* dx, int dadt, void* da, int64_t rows, int cols, float* part,
                            void* q, const float* scale, float* amax, int parts, int fmt, hipStream_t s) {
  if (cols % 8 || cols > 8 * 512 || !q || !scale || !amax || parts < 1) return (int)hipErrorInvalidValue;
  const Fp8Out q8{(uint8_t*)q, scale, amax, parts, fmt};
  switch ((cols + 511) / 512) {
    case 1: return bwd_dispatch<1>(dy, dydt, h, hdt, w, rstd, dres, dx, dadt, da, rows, cols, part, s, &q8);
    case 2: return bwd_dispatch<2>(dy, dydt, h, hdt, w, rstd, dres, dx, dadt, da, rows, cols, part, s, &q8);
    case 3: case 4: return bwd_dispatch<4>(dy, dydt, h, hdt, w, rstd, dres, dx, dadt, da, rows, cols, part, s, &q8);
    default: return bwd_dispatch<8>(dy, dydt, h, hdt, w, rstd, dres, dx, dadt, da, rows, cols, part, s, &q8);
  }
}

// out[c] += sum_r part[r][c]: the RMSNorm weight-gradient partials (one row per backward block)
// summed into the flat fp32 grad buffer in a fixed order (deterministic).  Latency-bound (a few MB):
// one workgroup per 64 columns, 16 row groups x 16 float4 column quads, 8 independent float4 loads
// in flight per thread, row groups combined through LDS.
__global__ void __launch_bounds__(256) colsum_add_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                         int rows, int cols) {
  __shared__ float4 red[16][17];
  const int q = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int c = blockIdx.x * 64 + q * 4;
  const bool ok = c < cols;  // cols % 4 == 0 (host check)
  float4 acc[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) {
    int r = rg;
    for (; r + 7 * 16 < rows; r += 8 * 16) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)(r + u * 16) * cols + c);
        acc[u].x += v.x; acc[u].y += v.y; acc[u].z += v.z; acc[u].w += v.w;
      }
    }
    for (; r < rows; r += 16) {
      const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)r * cols + c);
      acc[0].x += v.x; acc[0].y += v.y; acc[0].z += v.z; acc[0].w += v.w;
    }
  }
  float4 t = acc[0];
#pragma unroll
  for (int u = 1; u < 8; ++u) { t.x += acc[u].x; t.y += acc[u].y; t.z += acc[u].z; t.w += acc[u].w; }
  red[rg][q] = t;
  __syncthreads();
  if (rg == 0 && ok) {
    float4 s = red[0][q];
#pragma unroll
    for (int g = 1; g < 16; ++g) { s.x += red[g][q].x; s.y += red[g][q].y; s.z += red[g][q].z; s.w += red[g][q].w; }
    float4* o = reinterpret_cast<float4*>(out + c);
    float4 v = *o;
    v.x += s.x; v.y += s.y; v.z += s.z; v.w += s.w;
    *o = v;
  }
}

ND_API int nd_colsum_add(const float* part, float* out, int rows, int cols, hipStream_t s) {
  if (rows <= 0 || cols <= 0 || cols % 4 || ((uintptr_t)part & 15) || ((uintptr_t)out & 15))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(colsum_add_kernel, dim3((unsigned)((cols + 63) / 64)), dim3(256), 0, s, part, out, rows, cols);
  ND_LAUNCH_CHECK();
}
