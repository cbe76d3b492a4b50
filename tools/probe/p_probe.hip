// p_probe.hip -- standalone timing harness for the W = 1 partitioned count pass (C2 shape):
// a synthetic packed symbol stream (reads of 150 bases sampled from a 50 Mbp genome, each
// preceded by 8 break symbols, as the tokenizer emits a FASTA header), the C2 table
// geometry (-s 200000000), then WOps<1>::count_partitioned timed with HIP events, n times.
// Build: make -C tools/probe [EXP=n]; run under rocprofv3 --kernel-trace --stats for the
// per-kernel split.  Experiments (KC_EXP, kc_count_impl.h) are measurement-only builds.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../canonical-k-mer-hash-table_amd/csrc/kc_count_impl.h"

namespace kc {
template struct WOps<1>;
}
using namespace kc;

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));   \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

static __device__ uint64_t h64(uint64_t x) { return fmix64(x * 0x9E3779B97F4A7C15ULL + 0x632BE59BD9B4E019ULL); }

constexpr uint64_t RL = 150, HDR = 8, RS = RL + HDR;

__global__ void k_genome(uint64_t* g, uint64_t nw) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < nw) g[i] = h64(i ^ 0x1234);
}
__device__ uint32_t gsym(const uint64_t* g, uint64_t p) { return (uint32_t)(g[p >> 5] >> (62 - 2 * (p & 31))) & 3; }
__global__ void k_stream(const uint64_t* g, uint64_t glen, uint64_t nsym, uint64_t* pk, uint32_t* bk, uint64_t nw) {
    const uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (w >= nw) return;
    uint64_t v = 0;
    uint32_t b = 0;
    for (int j = 0; j < 32; j++) {
        const uint64_t p = w * 32 + j;
        uint32_t c = 0, br = 1;
        if (p < nsym) {
            const uint64_t r = p / RS, off = p % RS;
            if (off >= HDR) {
                const uint64_t pos = h64(r) % (glen - RL);
                c = gsym(g, pos + off - HDR);
                br = 0;
            }
        }
        v |= (uint64_t)c << (62 - 2 * j);
        b |= br << (31 - j);
    }
    pk[w] = v;
    bk[w] = b;
}

// bandwidth calibration: write / read / copy of n 16-byte items, grid-stride, uint4 per lane
__global__ void k_wr(uint4* p, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
__global__ void k_wr8(uint64_t* p, uint64_t n) {  // 8-byte stores (the scatter's store width)
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = i;
}
__global__ void k_rd(const uint4* p, uint64_t n, uint32_t* out) {
    uint32_t a = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        a ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (a == 0x12345678u) out[0] = a;
}
__global__ void k_cp(const uint4* s, uint4* d, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        d[i] = s[i];
}
// the level-1 store pattern without the sort: 2048 workgroups of 512 threads, each writing
// its own contiguous range in tiles of 8192 keys (16 coalesced 8-byte stores per thread per
// tile), with `work` dependent multiply-adds per key between tiles (0 = stores only;
// store = 0: compute only)
// ld: 0 no loads; 1 one load per thread per tile, used in the tile (issued after the
// previous tile's stores); 2 the same load prefetched one tile ahead and waited for before the
// stores
template <int LD>
__global__ __launch_bounds__(512, 4) void k_tilewr(uint64_t* out, uint64_t per, int work, int store,
                                                    const uint64_t* in) {
    const uint64_t base = blockIdx.x * per;
    uint64_t x = threadIdx.x * 0x9E3779B97F4A7C15ULL + blockIdx.x;
    uint64_t nx = LD == 2 ? in[(base >> 4) + threadIdx.x] : 0;
    for (uint64_t t = 0; t + 8192 <= per; t += 8192) {
        if (LD == 1) x ^= in[((base + t) >> 4) + threadIdx.x];
        if (LD == 2) {
            x ^= nx;
            nx = in[((base + t + 8192) >> 4) + threadIdx.x];
        }
        uint64_t v[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            for (int q = 0; q < work; q++) x = x * 0xff51afd7ed558ccdULL + (x >> 29);
            v[j] = x + j;
        }
        if (LD == 2) asm volatile("" : "+v"(nx));
        if (store) {
#pragma unroll
            for (int j = 0; j < 16; j++)
                if (store == 1 || ((threadIdx.x * 7 + j) & 3) != 0) out[base + t + j * 512 + threadIdx.x] = v[j];
        } else {
#pragma unroll
            for (int j = 0; j < 16; j++) x ^= v[j];
        }
    }
    if (!store && x == 42) out[0] = x;
}
// the level-1 segmented write pattern without the sort: each tile appends a run of `run`
// keys to each of F = 8192 / run bins (segment of bin b of this workgroup at
// (b * 2048 + blockIdx) * cap), 16 keys per thread per tile
__global__ __launch_bounds__(512, 4) void k_segwr(uint64_t* out, int tiles, int run, uint64_t cap) {
    const int F = 8192 / run;
    for (int t = 0; t < tiles; t++) {
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int i = q * 512 + threadIdx.x;
            const int b = i / run, rel = i - b * run;
            if (b < F) out[((uint64_t)b * 2048 + blockIdx.x) * cap + (uint64_t)t * run + rel] = i;
        }
    }
}
static void segwr() {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int run : {34, 32, 48, 64, 128, 33, 17, 16}) {
        const int tiles = 72, F = 8192 / run;
        const uint64_t cap = ((uint64_t)tiles * run + 15) / 16 * 16, n = (uint64_t)F * 2048 * cap;
        uint64_t* o;
        CK(hipMalloc(&o, n * 8));
        for (int rep = 0; rep < 2; rep++) {
            CK(hipEventRecord(e0, 0));
            k_segwr<<<2048, 512>>>(o, tiles, run, cap);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double bytes = 2048.0 * tiles * F * run * 8;
            printf("segwr run %3d (%3d bins): %.3f ms for %.2f GB = %.2f TB/s\n", run, F, ms, bytes / 1e9,
                   bytes / (ms * 1e-3) / 1e12);
        }
        CK(hipFree(o));
    }
}
static void tilewr() {
    const uint64_t per = 72 * 8192, n = 2048 * per;
    uint64_t* o;
    CK(hipMalloc(&o, n * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    uint64_t* in;
    CK(hipMalloc(&in, n / 16 * 8 + (1 << 20)));
    CK(hipMemset(in, 0, n / 16 * 8 + (1 << 20)));
    for (int ld : {0})
    for (int work : {0, 4})
        for (int store : {1, 2})
            for (int rep = 0; rep < 2; rep++) {
                CK(hipEventRecord(e0, 0));
                if (ld == 0) k_tilewr<0><<<2048, 512>>>(o, per, work, store, in);
                if (ld == 1) k_tilewr<1><<<2048, 512>>>(o, per, work, store, in);
                if (ld == 2) k_tilewr<2><<<2048, 512>>>(o, per, work, store, in);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                printf("tilewr ld %d work %d store %d: %.3f ms (%.2f TB/s of stores)\n", ld, work, store, ms,
                       store ? n * 8 / (ms * 1e-3) / 1e12 : 0.0);
            }
    CK(hipFree(o));
}
static void bw(uint64_t bytes) {
    uint4 *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    uint32_t* o;
    CK(hipMalloc(&o, 4));
    const uint64_t n = bytes / 16;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int grid : {1024, 4096, 16384}) {
        for (int rep = 0; rep < 3; rep++) {
            float t[4];
            for (int kk = 0; kk < 4; kk++) {
                CK(hipEventRecord(e0, 0));
                if (kk == 0) k_wr<<<grid, 256>>>(b, n);
                if (kk == 1) k_wr8<<<grid, 256>>>(reinterpret_cast<uint64_t*>(b), 2 * n);
                if (kk == 2) k_rd<<<grid, 256>>>(a, n, o);
                if (kk == 3) k_cp<<<grid, 256>>>(a, b, n);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&t[kk], e0, e1));
            }
            printf("bw grid %5d: write16 %.2f TB/s  write8 %.2f TB/s  read %.2f TB/s  copy %.2f TB/s (rd+wr)\n", grid,
                   bytes / (t[0] * 1e-3) / 1e12, bytes / (t[1] * 1e-3) / 1e12, bytes / (t[2] * 1e-3) / 1e12,
                   2 * bytes / (t[3] * 1e-3) / 1e12);
        }
    }
    CK(hipFree(a));
    CK(hipFree(b));
}


// level 1 without the LDS sort: every key goes straight from its register to its bin's segment
// at a position from a per-(workgroup, bin) LDS fill counter (no barriers, no tile in LDS);
// the partial lines of neighbouring keys of a bin are merged in L2.  F bins (uniform hash),
// tiles x 8192 keys per workgroup, 2048 workgroups of 512 threads.
// MODE 0: direct scattered 8-byte stores; 1: wave-local counting sort through LDS first (runs
// of a bin written by consecutive lanes), no workgroup barriers
template <int MODE>
__global__ __launch_bounds__(512, 4) void k_direct(uint64_t* out, int tiles, uint32_t F, uint64_t cap) {
    extern __shared__ uint32_t sm[];
    uint32_t* fill = sm;  // F counters
    for (uint32_t b = threadIdx.x; b < F; b += 512) fill[b] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t* wh = sm + F + wid * (2 * F + 2048 * 2);  // MODE 1: per wave: hist F, base F, keys 1024 x u64
    uint64_t* wk = reinterpret_cast<uint64_t*>(wh + 2 * F);
    uint64_t x = (blockIdx.x * 512ull + threadIdx.x) * 0x9E3779B97F4A7C15ULL;
    for (int t = 0; t < tiles; t++) {
        uint64_t v[16];
        uint32_t b[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            x = x * 0xff51afd7ed558ccdULL + 0x632BE59BD9B4E019ULL;
            v[j] = x;
            b[j] = __umulhi((uint32_t)(x >> 32), F);
        }
        if constexpr (MODE == 0) {
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const uint32_t pos = atomicAdd(&fill[b[j]], 1u);
                out[((uint64_t)b[j] * 2048 + blockIdx.x) * cap + pos] = v[j];
            }
        } else {
            for (uint32_t i = lane; i < F; i += 64) wh[i] = 0;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            uint32_t rk[16];
#pragma unroll
            for (int j = 0; j < 16; j++) rk[j] = atomicAdd(&wh[b[j]], 1u);
            // wave scan of the F counts (F / 64 per lane) + one fill atomic per (wave, bin)
            uint32_t per = (F + 63) / 64, lo = lane * per, sum = 0;
            for (uint32_t i = lo; i < lo + per && i < F; i++) sum += wh[i];
            const uint32_t incl = wave_incl_sum(sum);
            uint32_t run = incl - sum;
            for (uint32_t i = lo; i < lo + per && i < F; i++) {
                const uint32_t h = wh[i];
                wh[F + i] = run;  // start of bin i in the wave's sorted block
                wh[i] = h ? atomicAdd(&fill[i], h) : 0;  // destination of its first key
                run += h;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
            for (int j = 0; j < 16; j++) wk[wh[F + b[j]] + rk[j]] = v[j] ^ ((uint64_t)b[j] << 48);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const uint32_t i = q * 64 + lane;
                const uint64_t key = wk[i];
                const uint32_t bb = (uint32_t)(key >> 48) & 0xFFFF;  // (probe: the bin rides in the key)
                const uint32_t pos = wh[bb] + (i - wh[F + bb]);
                out[((uint64_t)bb * 2048 + blockIdx.x) * cap + pos] = key;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        }
    }
}
static void direct() {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (uint32_t F : {240u, 120u, 480u}) {
        const int tiles = 72;
        const uint64_t cap = ((uint64_t)tiles * 8192 / F * 5 / 4 + 15) / 16 * 16, n = (uint64_t)F * 2048 * cap;
        uint64_t* o;
        CK(hipMalloc(&o, n * 8));
        for (int mode = 0; mode < 2; mode++) {
            const size_t sm = mode ? (F + 8 * (2 * F + 4096)) * 4 : F * 4;
            if (mode) CK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_direct<1>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
            for (int rep = 0; rep < 2; rep++) {
                CK(hipEventRecord(e0, 0));
                if (mode == 0) k_direct<0><<<2048, 512, sm>>>(o, tiles, F, cap);
                else k_direct<1><<<2048, 512, sm>>>(o, tiles, F, cap);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double bytes = 2048.0 * tiles * 8192 * 8;
                printf("direct mode %d F %u: %.3f ms for %.2f GB = %.2f TB/s\n", mode, F, ms, bytes / 1e9,
                       bytes / (ms * 1e-3) / 1e12);
            }
        }
        CK(hipFree(o));
    }
}

int main(int argc, char** argv) {
    if (argc > 1 && argv[1][0] == 'b') {
        bw(9600000000ULL);
        return 0;
    }
    if (argc > 1 && argv[1][0] == 't') {
        tilewr();
        return 0;
    }
    if (argc > 1 && argv[1][0] == 'd') {
        direct();
        return 0;
    }
    if (argc > 1 && argv[1][0] == 's') {
        segwr();
        return 0;
    }
    const uint64_t reads = argc > 1 ? strtoull(argv[1], 0, 10) : 10000000ULL;
    const int iters = argc > 2 ? atoi(argv[2]) : 5;
    const int k = 31;
    const uint64_t slots = 200000000ULL, glen = 50000000ULL;
    const uint64_t M = reads * RS, nw = M / 32 + 4;
    uint64_t *g, *pk;
    uint32_t* bk;
    CK(hipMalloc(&g, (glen / 32 + 1) * 8));
    CK(hipMalloc(&pk, nw * 8));
    CK(hipMalloc(&bk, nw * 4));
    k_genome<<<(glen / 32 + 256) / 256, 256>>>(g, glen / 32 + 1);
    k_stream<<<(nw + 255) / 256, 256>>>(g, glen, M, pk, bk, nw);
    CK(hipDeviceSynchronize());
    // table geometry (kc_api.cpp alloc_table)
    uint64_t want = slots + slots / 4;
    const uint64_t buckets = (want + 7) / 8, regions = (buckets + BPR - 1) / BPR;
    int rbits = 0;
    while ((1ULL << rbits) < regions) rbits++;
    const int f1bits = std::min(10, (rbits + 1) / 2);
    TableView t{};
    t.f2bits = rbits - f1bits;
    t.F2 = 1u << t.f2bits;
    t.F1 = (uint32_t)((regions + t.F2 - 1) / t.F2);
    if ((uint64_t)t.F1 * t.F2 >= 49152 && (uint64_t)t.F1 * t.F2 < 65536) t.F1 = (65536 + t.F2 - 1) / t.F2;  // alloc_table
    t.R = (uint64_t)t.F1 * t.F2;
    t.nbuckets = t.R * BPR;
    t.W = 1;
    t.S = 8;
    CK(hipMalloc(&t.buckets, t.nbuckets * 128));
    // partition buffers (kc_api.cpp ensure_part_geo, segmented)
    PartBufs pb{};
    const uint64_t tile = (uint64_t)COUNT_THREADS * run_width(1);
    pb.nblk1 = (uint32_t)std::min<uint64_t>(2048, (M + tile - 1) / tile);
    pb.B2 = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(64, 2048 / t.F1));
    auto capacity = [](double e) { return ((uint64_t)std::ceil(e + 8.0 * std::sqrt(e) + 32.0) + 7) / 8 * 8; };
    const uint64_t t1 = p1_tile(1);
    const uint64_t per1 = ((M + pb.nblk1 - 1) / pb.nblk1 + t1 - 1) / t1 * t1;
    const uint64_t nseg = (pb.nblk1 + pb.B2 - 1) / pb.B2;
    pb.cap1 = capacity((double)per1 / t.F1);
    pb.cap2 = capacity((double)nseg * per1 / t.F1 / t.F2);
    const uint64_t n1 = (uint64_t)t.F1 * 2048, n2 = t.R * pb.B2;
    CK(hipMalloc(&pb.hist1, n1 * 4));
    CK(hipMalloc(&pb.off1, (n1 + 1) * 8));
    CK(hipMalloc(&pb.hist2, n2 * 4));
    CK(hipMalloc(&pb.off2, (n2 + 1) * 8));
    CK(hipMalloc(&pb.bsum, ((std::max(n1, n2) + 4095) / 4096 + 2) * 8));
    pb.spill_cap = std::max<uint64_t>(1 << 16, M / 8);
    const uint64_t need1 = std::max<uint64_t>(M, (uint64_t)t.F1 * pb.nblk1 * pb.cap1);
    const uint64_t need2 = std::max<uint64_t>(M, t.R * pb.B2 * pb.cap2);
    CK(hipMalloc(&pb.keys1, std::max(need1, pb.spill_cap * 2) * 8));
    CK(hipMalloc(&pb.keys2, std::max(need2, pb.spill_cap * 2) * 8));
    CK(hipMalloc(&pb.spill, pb.spill_cap * 2 * 8));
    DevCounters* ctr;
    CK(hipMalloc(&ctr, sizeof(DevCounters)));
    printf("reads %llu symbols %llu R %llu F1 %u F2 %u nblk1 %u B2 %u cap1 %llu cap2 %llu\n", (unsigned long long)reads,
           (unsigned long long)M, (unsigned long long)t.R, t.F1, t.F2, pb.nblk1, pb.B2, (unsigned long long)pb.cap1,
           (unsigned long long)pb.cap2);
    PackedView sv{pk, bk};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t expect = reads * (RL - k + 1);
    for (int it = 0; it < iters; it++) {
        DevCounters h{};
        h.stream_len = M;
        CK(hipMemcpy(ctr, &h, sizeof(h), hipMemcpyHostToDevice));
        CK(hipEventRecord(e0, 0));
        CK(WOps<1>::count_partitioned(sv, k, 0, t, BloomView{}, ctr, pb, 1, 0, PH_ALL));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(&h, ctr, sizeof(h), hipMemcpyDeviceToHost));
        printf("iter %d: %.3f ms  windows %llu (expect %llu) inserted %llu overflow %llu part_overflow %llu "
               "spilled %llu heavy %llu -> %.1f G windows/s\n",
               it, ms, h.windows, (unsigned long long)expect, h.inserted, h.overflow, h.part_overflow, h.spill_n,
               h.heavy_n, expect / (ms * 1e-3) / 1e9);
    }
#if KC_STAMP
    {  // one more pass with the phase stamps cleared first
        static unsigned long long h[6144 * 8];
        memset(h, 0, sizeof(h));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), h, sizeof(h)));
        DevCounters hc{};
        hc.stream_len = M;
        CK(hipMemcpy(ctr, &hc, sizeof(hc), hipMemcpyHostToDevice));
        CK(WOps<1>::count_partitioned(sv, k, 0, t, BloomView{}, ctr, pb, 1, 0, PH_ALL));
        CK(hipDeviceSynchronize());
        CK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_stamp), sizeof(h)));
        const char* ph[8] = {"extraction+combine", "rank atomics", "barrier 1", "scan+barrier 2",
                             "placement+setup", "barrier 3", "write-out", "-"};
        const int nb[3] = {(int)pb.nblk1, (int)(t.F1 * pb.B2), 2048};
        for (int part = 0; part < 3; part++) {
            if (part == 2) {  // level 3: 61440 workgroups folded onto 2048 slots; phases 0-3
                double a[4] = {0, 0, 0, 0}, tot = 0;
                for (int b = 0; b < 2048; b++)
                    for (int i = 0; i < 4; i++) a[i] += h[(2 * 2048 + b) * 8 + i];
                const char* p3[4] = {"region init", "items (loads + inserts)", "barrier", "write-back"};
                for (int i = 0; i < 4; i++) { a[i] /= (double)t.R; tot += a[i]; }
                printf("stamps k_p3 (cycles per workgroup):");
                for (int i = 0; i < 4; i++) printf(" [%s] %.0f (%.1f%%)", p3[i], a[i], 100 * a[i] / tot);
                printf(" total %.0f\n", tot);
                continue;
            }
            double tot = 0, a[8];
            for (int i = 0; i < 8; i++) {
                a[i] = 0;
                for (int b = 0; b < std::min(nb[part], 2048); b++) a[i] += h[(part * 2048 + b) * 8 + i];
                a[i] /= std::min(nb[part], 2048);
                tot += a[i];
            }
            printf("stamps %s (cycles per workgroup, wave 0):", part ? "k_p2f" : "k_p1");
            for (int i = 0; i < 8; i++) printf(" [%s] %.0f (%.1f%%)", ph[i], a[i], 100 * a[i] / tot);
            printf(" total %.0f\n", tot);
        }
    }
#endif
    return 0;
}
