// kc_util.hip -- small device helpers behind the C ABI's test hooks: the device XXH64
// of the reference-layout Bloom passes (kc_common.h xxh64_u64) over host-given inputs.
#include "kc_common.h"

namespace kc {

__global__ __launch_bounds__(256) void k_xxh64(const uint64_t* __restrict__ v, const uint64_t* __restrict__ seed,
                                               uint64_t n, uint64_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = xxh64_u64(v[i], seed[i]);
}

hipError_t launch_xxh64(const uint64_t* v, const uint64_t* seed, uint64_t n, uint64_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_xxh64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, v, seed, n, out);
    return hipGetLastError();
}

}  // namespace kc
