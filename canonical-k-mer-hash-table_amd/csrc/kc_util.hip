// kc_util.hip -- small device helpers: the device XXH64 of the reference-layout Bloom
// passes (kc_common.h xxh64_u64) over host-given inputs (test hook), the chunk checksum of
// the partition reuse, and the sharded Bloom filter's merge and filter-2 bit count.
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

// Checksum of the chunks' bytes: the sum over every aligned 8-byte word w overlapping a
// chunk of fmix64(w's chunk bytes + its address * C), bytes outside the chunk masked.
// Two passes over one image compare their sums (kc_api.cpp level-1 reuse).
constexpr int CK_T = 256, CK_PER = 32;  // words per thread
constexpr int CK_SLOTS = 64;            // partial sums (the caller adds them)
__global__ __launch_bounds__(CK_T) void k_checksum(const uint8_t* __restrict__ src, const ChunkDesc* __restrict__ ch,
                                                   unsigned long long* __restrict__ out) {
    const ChunkDesc d = ch[blockIdx.y];
    const uint64_t a0 = (reinterpret_cast<uint64_t>(src) + d.src_off) & ~7ull;  // first aligned word
    const uint64_t end = reinterpret_cast<uint64_t>(src) + d.src_off + d.len;
    const uint64_t beg = reinterpret_cast<uint64_t>(src) + d.src_off;
    unsigned long long h = 0;
#pragma unroll
    for (int q = 0; q < CK_PER; q++) {
        const uint64_t a = a0 + 8 * ((uint64_t)blockIdx.x * CK_T * CK_PER + (uint64_t)q * CK_T + threadIdx.x);
        if (a >= end) continue;
        uint64_t v = *reinterpret_cast<const uint64_t*>(a);
        if (a < beg) v &= ~0ull << (8 * (beg - a));              // little-endian: low bytes first
        if (a + 8 > end) v &= ~0ull >> (8 * (a + 8 - end));
        h += fmix64(v + (a - reinterpret_cast<uint64_t>(src)) * 0x9E3779B97F4A7C15ull + blockIdx.y);
    }
    for (int o = 32; o >= 1; o >>= 1) h += __shfl_xor(h, o, 64);
    __shared__ unsigned long long s_h[CK_T / 64];
    if ((threadIdx.x & 63) == 0) s_h[threadIdx.x >> 6] = h;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < CK_T / 64; w++) t += s_h[w];
        // one add per workgroup, spread over CK_SLOTS words (one word takes ~90 adds per us)
        if (t) atomicAdd(out + ((blockIdx.x + blockIdx.y * 7) % CK_SLOTS), t);
    }
}

hipError_t launch_checksum(const uint8_t* src, const ChunkDesc* d_chunks, int n_chunks, uint64_t max_len,
                           unsigned long long* out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, CK_SLOTS * sizeof(unsigned long long), s);
    if (e != hipSuccess || n_chunks == 0) return e;
    const uint64_t words = max_len / 8 + 2, per = (uint64_t)CK_T * CK_PER;
    hipLaunchKernelGGL(k_checksum, dim3((unsigned)((words + per - 1) / per), (unsigned)n_chunks), dim3(CK_T), 0, s, src,
                       d_chunks, out);
    return hipGetLastError();
}

// Sharded Bloom filter (kc_bloom_merge_device).  The ranks' filters after their own Bloom
// passes are combined so that the gate passes every k-mer the reference's one filter would
// pass for count >= 2 (double_bloomfilter.hpp:233-246 insertion_process): a k-mer seen twice
// on one rank has its filter-2 bits set there (OR), one seen on two ranks has its filter-1
// bits set in two copies.  Blocked layout: thread = word w < 8 of a block, filter 1 at w,
// filter 2 at w + 8.  Reference layout: thread = word, filter 1 = even bits, filter 2 = odd.
__global__ __launch_bounds__(256) void k_bloom_merge(const uint32_t* __restrict__ parts, uint32_t nparts, uint64_t n,
                                                     int blocked, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t once = 0, twice = 0, f2 = 0;
    if (blocked) {
        if (i >= n / 2) return;
        const uint64_t a = (i >> 3) * 16 + (i & 7);
        for (uint32_t p = 0; p < nparts; p++) {
            const uint32_t x = parts[p * n + a];
            twice |= once & x;
            once |= x;
            f2 |= parts[p * n + a + 8];
        }
        out[a] = once;
        out[a + 8] = f2 | twice;
    } else {
        if (i >= n) return;
        for (uint32_t p = 0; p < nparts; p++) {
            const uint32_t x = parts[p * n + i];
            const uint32_t x1 = x & 0x55555555u;
            twice |= once & x1;
            once |= x1;
            f2 |= x & 0xAAAAAAAAu;
        }
        out[i] = once | f2 | (twice << 1);
    }
}

hipError_t launch_bloom_merge(const uint32_t* parts, uint32_t nparts, uint64_t n, int blocked, uint32_t* out,
                              hipStream_t s) {
    const uint64_t threads = blocked ? n / 2 : n;
    if (threads == 0) return hipSuccess;
    hipLaunchKernelGGL(k_bloom_merge, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, parts, nparts, n,
                       blocked, out);
    return hipGetLastError();
}

constexpr int PC_PER = 16;  // words per thread
__global__ __launch_bounds__(256) void k_bloom_popcount2(const uint32_t* __restrict__ w, uint64_t n, int blocked,
                                                         unsigned long long* __restrict__ out) {
    unsigned long long c = 0;
#pragma unroll
    for (int q = 0; q < PC_PER; q++) {
        const uint64_t i = ((uint64_t)blockIdx.x * PC_PER + q) * 256 + threadIdx.x;
        if (i >= n) break;
        const uint32_t x = w[i];
        c += blocked ? ((i & 15) >= 8 ? __popc(x) : 0) : __popc(x & 0xAAAAAAAAu);
    }
    for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
    __shared__ unsigned long long s_c[4];
    if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = s_c[0] + s_c[1] + s_c[2] + s_c[3];
        if (t) atomicAdd(out + blockIdx.x % CK_SLOTS, t);
    }
}

hipError_t launch_bloom_popcount2(const uint32_t* words, uint64_t n, int blocked, unsigned long long* out,
                                  hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, CK_SLOTS * sizeof(unsigned long long), s);
    if (e != hipSuccess || n == 0) return e;
    const uint64_t per = 256ull * PC_PER;
    hipLaunchKernelGGL(k_bloom_popcount2, dim3((unsigned)((n + per - 1) / per)), dim3(256), 0, s, words, n, blocked,
                       out);
    return hipGetLastError();
}

// deferred level 3 (kc_api.cpp run_deferred): a batch whose segments overflowed holds its
// part_overflow aside while the group's level 3 inserts the other batches (k_p3 skips on the
// flag), then gets it back for its tail (the exact pipeline redoes that batch)
__global__ void k_hold_overflow(DevCounters* ctr, int restore) {
    if (restore) {
        ctr->part_overflow = ctr->held_overflow;
        ctr->held_overflow = 0;
    } else {
        ctr->held_overflow = ctr->part_overflow;
        ctr->part_overflow = 0;
    }
}

hipError_t launch_hold_overflow(DevCounters* ctr, int restore, hipStream_t s) {
    hipLaunchKernelGGL(k_hold_overflow, dim3(1), dim3(1), 0, s, ctr, restore);
    return hipGetLastError();
}

}  // namespace kc
