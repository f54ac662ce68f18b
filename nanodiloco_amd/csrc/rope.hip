// Rotary position embedding, in place on the packed q|k|v projection output (K4).
//
// Layout: rows = B*T tokens, each row = [q heads (nh*hd) | k heads (nkv*hd) | v heads (nkv*hd)],
// row stride `ld` elements.  Half-split (HF rotate_half) convention: element i pairs with
// i + hd/2.  Tables are fp32 [T, hd] (cat(freqs, freqs)), so only the first half is read.
// One thread rotates 4 pairs (8-B bf16 / 16-B fp32 vector accesses); math in fp32, one rounding.
// inverse=1 applies R(-theta): the exact backward of the forward rotation (used on dq|dk).
#include "common.h"

using namespace nd;

template <int DT>
__global__ void __launch_bounds__(256) rope_kernel(void* __restrict__ qkv, const float* __restrict__ cosT,
                                                   const float* __restrict__ sinT, int64_t rows, int T, int nheads,
                                                   int hd, int ld, int inverse) {
  const int half = hd >> 1;
  const int q4 = half >> 2;  // groups of 4 pairs per head
  const int64_t total = rows * nheads * q4;
  for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < total; it += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(it % q4);
    const int64_t rh = it / q4;
    const int head = (int)(rh % nheads);
    const int64_t row = rh / nheads;
    const int t = (int)(row % T);
    const int i0 = g * 4;
    const float4 c = *reinterpret_cast<const float4*>(cosT + (int64_t)t * hd + i0);
    float4 sn = *reinterpret_cast<const float4*>(sinT + (int64_t)t * hd + i0);
    if (inverse) { sn.x = -sn.x; sn.y = -sn.y; sn.z = -sn.z; sn.w = -sn.w; }
    const int64_t base = row * ld + (int64_t)head * hd + i0;
    float x1[4], x2[4];
    if (DT == BF16) {
      bf16_t* p = reinterpret_cast<bf16_t*>(qkv);
      uint2 a = *reinterpret_cast<const uint2*>(p + base);
      uint2 b = *reinterpret_cast<const uint2*>(p + base + half);
      x1[0] = lo_bf(a.x); x1[1] = hi_bf(a.x); x1[2] = lo_bf(a.y); x1[3] = hi_bf(a.y);
      x2[0] = lo_bf(b.x); x2[1] = hi_bf(b.x); x2[2] = lo_bf(b.y); x2[3] = hi_bf(b.y);
    } else {
      float* p = reinterpret_cast<float*>(qkv);
      float4 a = *reinterpret_cast<const float4*>(p + base);
      float4 b = *reinterpret_cast<const float4*>(p + base + half);
      x1[0] = a.x; x1[1] = a.y; x1[2] = a.z; x1[3] = a.w;
      x2[0] = b.x; x2[1] = b.y; x2[2] = b.z; x2[3] = b.w;
    }
    const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
    float y1[4], y2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      y1[j] = x1[j] * cc[j] - x2[j] * ss[j];
      y2[j] = x2[j] * cc[j] + x1[j] * ss[j];
    }
    if (DT == BF16) {
      bf16_t* p = reinterpret_cast<bf16_t*>(qkv);
      *reinterpret_cast<uint2*>(p + base) = make_uint2(pack2(y1[0], y1[1]), pack2(y1[2], y1[3]));
      *reinterpret_cast<uint2*>(p + base + half) = make_uint2(pack2(y2[0], y2[1]), pack2(y2[2], y2[3]));
    } else {
      float* p = reinterpret_cast<float*>(qkv);
      *reinterpret_cast<float4*>(p + base) = make_float4(y1[0], y1[1], y1[2], y1[3]);
      *reinterpret_cast<float4*>(p + base + half) = make_float4(y2[0], y2[1], y2[2], y2[3]);
    }
  }
}

// Rotates the first (nh + nkv) heads of every row (q and k); v is untouched.
ND_API int nd_rope_inplace(void* qkv, int dt, const float* cosT, const float* sinT, int64_t rows, int T, int nh,
                           int nkv, int hd, int ld, int inverse, hipStream_t s) {
  if (hd % 8) return (int)hipErrorInvalidValue;
  const int nheads = nh + nkv;
  const int64_t total = rows * nheads * (hd / 8);
  int64_t blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (dt == BF16)
    hipLaunchKernelGGL(rope_kernel<BF16>, dim3((unsigned)blocks), dim3(256), 0, s, qkv, cosT, sinT, rows, T, nheads,
                       hd, ld, inverse);
  else
    hipLaunchKernelGGL(rope_kernel<F32>, dim3((unsigned)blocks), dim3(256), 0, s, qkv, cosT, sinT, rows, T, nheads,
                       hd, ld, inverse);
  ND_LAUNCH_CHECK();
}
