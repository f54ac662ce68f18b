// Hardware-semantics probes (GPU tests only): what a gfx950 LDS instruction returns for given per-lane
// addresses, so kernels that depend on an undocumented layout pin it with a test (tests/test_probe_gpu.py).
#include "common.h"

namespace {
typedef int v2i __attribute__((ext_vector_type(2)));

// one wave: LDS <- in[0, 4096); lane l issues ds_read_b64_tr_b8 at byte offset addr[l]; out[l] = the 8 bytes
__global__ void __launch_bounds__(64) probe_tr8_kernel(const uint8_t* __restrict__ in, const int* __restrict__ addr,
                                                       int* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t s[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) s[i] = in[i];
  __syncthreads();
  const int a = addr[threadIdx.x] & 4088;
  const v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((v2i __attribute__((address_space(3)))*)(s + a));
  out[threadIdx.x * 2] = r[0];
  out[threadIdx.x * 2 + 1] = r[1];
}
}  // namespace

ND_API int nd_probe_tr8(const void* in, const int* addr, int* out, hipStream_t s) {
  hipLaunchKernelGGL(probe_tr8_kernel, dim3(1), dim3(64), 0, s, (const uint8_t*)in, addr, out);
  ND_LAUNCH_CHECK();
}
