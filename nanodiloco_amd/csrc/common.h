// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernels.
// Wave = 64 lanes everywhere; bf16 is stored as raw uint16 and converted with the native
// v_cvt_pk_bf16_f32 (via clang's __bf16) -- NaN-preserving, RNE.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ND_API extern "C" __attribute__((visibility("default")))

namespace nd {

constexpr int WAVE = 64;
enum DType : int { F32 = 0, BF16 = 1 };

typedef uint16_t bf16_t;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));   // MFMA A/B fragment (8 bf16)
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 pair (RNE): one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{a, b}), bf16x2_t));
}
// logistic sigmoid with the hardware reciprocal (v_rcp_f32, 1 ulp) and exponential: 4 VALU.  A plain
// `1.f / (1.f + e)` compiles to the IEEE division sequence (div_scale / rcp / 4 fma / div_fmas / div_fixup,
// 11 VALU), which made up half of the fused SwiGLU-backward GEMM epilogue.  x -> -inf: rcp(inf) = 0.
__device__ __forceinline__ float fast_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float lo_bf(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// Load / store 8 consecutive elements of either dtype as fp32 (16-B or 32-B vector access).
template <int DT> struct Vec8;
template <> struct Vec8<F32> {
  __device__ __forceinline__ static void load(const void* p, int64_t i, float* v) {
    const float4* q = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p) + i);
    float4 a = q[0], b = q[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ static void store(void* p, int64_t i, const float* v) {
    float4* q = reinterpret_cast<float4*>(reinterpret_cast<float*>(p) + i);
    q[0] = make_float4(v[0], v[1], v[2], v[3]);
    q[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};
template <> struct Vec8<BF16> {
  __device__ __forceinline__ static void load(const void* p, int64_t i, float* v) {
    uint4 a = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(p) + i);
    v[0] = lo_bf(a.x); v[1] = hi_bf(a.x); v[2] = lo_bf(a.y); v[3] = hi_bf(a.y);
    v[4] = lo_bf(a.z); v[5] = hi_bf(a.z); v[6] = lo_bf(a.w); v[7] = hi_bf(a.w);
  }
  __device__ __forceinline__ static void store(void* p, int64_t i, const float* v) {
    uint4 a;
    a.x = pack2(v[0], v[1]); a.y = pack2(v[2], v[3]); a.z = pack2(v[4], v[5]); a.w = pack2(v[6], v[7]);
    *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(p) + i) = a;
  }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x = NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NT == 64) return v;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  return t;
}

// XCD-aware block remap (bijective for any grid size): consecutive logical tiles land on the
// same XCD's L2.  blocks b and b+8 share an XCD under round-robin dispatch (speed only).
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int q = nblocks / 8, r = nblocks % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// ---- OCP fp8 (gfx950 v_cvt_pk_fp8_f32 / v_cvt_pk_bf8_f32: e4m3fn / e5m2, RNE), saturating
template <int FMT>  // 0: e4m3 (max 448), 1: e5m2 (max 57344)
__device__ __forceinline__ uint32_t cvt4(float a, float b, float c, float d) {
  constexpr float FMAX = FMT == 0 ? 448.f : 57344.f;
  a = fminf(fmaxf(a, -FMAX), FMAX);
  b = fminf(fmaxf(b, -FMAX), FMAX);
  c = fminf(fmaxf(c, -FMAX), FMAX);
  d = fminf(fmaxf(d, -FMAX), FMAX);
  int r;
  if (FMT == 0) {
    r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  } else {
    r = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
    r = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, r, true);
  }
  return (uint32_t)r;
}

// Fused fp8 side output of a bf16-producing kernel (the fp8 inner step's operand quantisation
// folded into the producer): q[i] = fp8(bf16(v[i]) * scale), amax of |bf16(v[i])| -- bitwise the
// separate nd_fp8_cast pass over the bf16 tensor.  q == nullptr: no side output.
struct Fp8Out {
  uint8_t* q;
  const float* scale;  // device scalar (delayed scaling: known before the producer runs)
  float* amax;         // `parts` partial maxima (float bits as ordered ints), block b -> b % parts
  int parts;
  int fmt;             // 0 e4m3, 1 e5m2
};

// v: 8 fp32 values already rounded to bf16; writes 8 fp8 bytes at q + off, folds |v| into amax
__device__ __forceinline__ void fp8_put8(const Fp8Out& f, int64_t off, const float* v, float& amax) {
  const float sc = f.scale[0];
#pragma unroll
  for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[j]));
  uint2 o;
  if (f.fmt == 0) {
    o.x = cvt4<0>(v[0] * sc, v[1] * sc, v[2] * sc, v[3] * sc);
    o.y = cvt4<0>(v[4] * sc, v[5] * sc, v[6] * sc, v[7] * sc);
  } else {
    o.x = cvt4<1>(v[0] * sc, v[1] * sc, v[2] * sc, v[3] * sc);
    o.y = cvt4<1>(v[4] * sc, v[5] * sc, v[6] * sc, v[7] * sc);
  }
  *reinterpret_cast<uint2*>(f.q + off) = o;
}

// bf16 store of 8 values and their fp8 side output from the SAME packed bf16 words: the rounded values
// are unpacked (one shift / and each) instead of rounded a second time.  sc: the side output's scale,
// read once per kernel by the caller.  Bitwise Vec8<BF16>::store + round_bf16x8 + fp8_put8.
template <int FMT>
__device__ __forceinline__ void put8_bf16_q_t(void* y, int64_t i, const float* v, uint8_t* q, float sc, float& amax) {
  uint4 a;
  a.x = pack2(v[0], v[1]); a.y = pack2(v[2], v[3]); a.z = pack2(v[4], v[5]); a.w = pack2(v[6], v[7]);
  *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(y) + i) = a;
  const float r[8] = {lo_bf(a.x), hi_bf(a.x), lo_bf(a.y), hi_bf(a.y), lo_bf(a.z), hi_bf(a.z), lo_bf(a.w), hi_bf(a.w)};
#pragma unroll
  for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(r[j]));
  uint2 o;
  o.x = cvt4<FMT>(r[0] * sc, r[1] * sc, r[2] * sc, r[3] * sc);
  o.y = cvt4<FMT>(r[4] * sc, r[5] * sc, r[6] * sc, r[7] * sc);
  *reinterpret_cast<uint2*>(q + i) = o;
}
__device__ __forceinline__ void put8_bf16_q(void* y, int64_t i, const float* v, const Fp8Out& f, float sc, float& amax) {
  if (f.fmt == 0) put8_bf16_q_t<0>(y, i, v, f.q, sc, amax);
  else put8_bf16_q_t<1>(y, i, v, f.q, sc, amax);
}

__device__ __forceinline__ void round_bf16x8(float* v) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = bf2f(f2bf(v[j]));
}

// Block-wide amax -> one atomicMax into a partial slot.  Every thread of the block must call it
// (it contains barriers); NT = block size.  Non-negative floats order like their int bits.
template <int NT>
__device__ __forceinline__ void block_amax_commit(float amax, float* amax_out, int parts) {
  __shared__ float red_amax[NT / 64];
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red_amax[threadIdx.x >> 6] = amax;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = red_amax[0];
#pragma unroll
    for (int i = 1; i < NT / 64; ++i) m = fmaxf(m, red_amax[i]);
    atomicMax(reinterpret_cast<int*>(amax_out + blockIdx.x % parts), __float_as_int(m));
  }
}

// Four LDS-DMA wave-instructions (64 lanes x 16 B each) from per-lane byte offsets v0..v3 into LDS lds, lds + ST,
// lds + 2 ST, lds + 3 ST: m0 is saved / restored once per burst and stepped with one s_add per piece (the
// compiler reserves m0, so every asm that writes it must restore it; SCC is declared clobbered).  The one wait
// state between an m0 write and the LDS-DMA that reads it is the s_nop.  FLAT-global form (SGPR base, no range
// check) and buffer form (range-checked V#: lanes past its record count read nothing).
#ifndef ND_DMA_BURST
#define ND_DMA_BURST 1
#endif
template <uint32_t ST>
__device__ __forceinline__ void gdma4(const void* base, uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %5\n\t"
      "s_add_u32 m0, m0, %7\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %5\n\t"
      "s_add_u32 m0, m0, %7\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %3, %5\n\t"
      "s_add_u32 m0, m0, %7\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %4, %5\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "v"(v1), "v"(v2), "v"(v3), "s"(base), "s"(lds), "i"(ST)
      : "memory", "scc");
}
template <uint32_t ST>
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t r, uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3,
                                     uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %5, 0 offen lds\n\t"
      "s_add_u32 m0, m0, %7\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %5, 0 offen lds\n\t"
      "s_add_u32 m0, m0, %7\n\ts_nop 0\n\tbuffer_load_dwordx4 %3, %5, 0 offen lds\n\t"
      "s_add_u32 m0, m0, %7\n\ts_nop 0\n\tbuffer_load_dwordx4 %4, %5, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(v0), "v"(v1), "v"(v2), "v"(v3), "s"(r), "s"(lds), "i"(ST)
      : "memory", "scc");
}

}  // namespace nd

#define ND_LAUNCH_CHECK() return (int)hipGetLastError()
