// pmc_calib -- PMC byte calibration for the store / load widths the engine uses:
// each kernel moves a known number of bytes with one access shape, coalesced, lane i on record i;
// rocprofv3 --pmc WRITE_SIZE / FETCH_SIZE of each dispatch against those bytes gives the counter's
// unit for that shape (MI355X_MICROARCH.md: exact only for 16-B streaming stores; FETCH_SIZE = 1/2
// of a 16-B streaming read).  Shapes: 16-B (uint4), 12-B (uint3: Rec12 records), 8-B (one-word keys),
// 6-B (StoreRec6: a dword + a short per record, two records per three dwords), 1-B (k_synth's FASTA
// bytes).  Prints one line per kernel: name, records, bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void cal_store16(uint4* o, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        o[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
__global__ void cal_store12(uint3* o, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        o[i] = make_uint3((uint32_t)i, 1, 2);
}
__global__ void cal_store8(uint64_t* o, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) o[i] = i;
}
__global__ void cal_store6(uint32_t* o, uint64_t n) {  // StoreRec6's two stores per record
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        uint32_t* q = o + (i >> 1) * 3;
        q[i & 1] = (uint32_t)i;
        reinterpret_cast<uint16_t*>(q + 2)[i & 1] = (uint16_t)i;
    }
}
__global__ void cal_store1(uint8_t* o, uint64_t n) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) o[i] = (uint8_t)i;
}
__global__ void cal_load16(const uint4* in, uint64_t n, uint32_t* sink) {
    uint32_t a = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = in[i];
        a ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (a == 0x12345678u) sink[0] = a;
}
__global__ void cal_load12(const uint3* in, uint64_t n, uint32_t* sink) {
    uint32_t a = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint3 v = in[i];
        a ^= v.x ^ v.y ^ v.z;
    }
    if (a == 0x12345678u) sink[0] = a;
}
__global__ void cal_load8(const uint64_t* in, uint64_t n, uint32_t* sink) {
    uint64_t a = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) a ^= in[i];
    if (a == 0x12345678u) sink[0] = (uint32_t)a;
}

int main() {
    const uint64_t bytes = 3ull << 30;  // past the 256 MiB Infinity Cache
    uint8_t* buf = nullptr;
    uint32_t* sink = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess) return 1;
    const dim3 g(4096), b(256);
    auto run = [&](const char* name, uint64_t recs, uint64_t moved, auto launch) {
        launch();
        if (hipDeviceSynchronize() != hipSuccess) { std::printf("%s failed\n", name); return; }
        std::printf("%s records=%llu bytes=%llu\n", name, (unsigned long long)recs, (unsigned long long)moved);
    };
    uint64_t n;
    n = bytes / 16; run("cal_store16", n, n * 16, [&] { hipLaunchKernelGGL(cal_store16, g, b, 0, 0, (uint4*)buf, n); });
    n = bytes / 12; run("cal_store12", n, n * 12, [&] { hipLaunchKernelGGL(cal_store12, g, b, 0, 0, (uint3*)buf, n); });
    n = bytes / 8;  run("cal_store8", n, n * 8, [&] { hipLaunchKernelGGL(cal_store8, g, b, 0, 0, (uint64_t*)buf, n); });
    n = bytes / 6 / 2 * 2; run("cal_store6", n, n * 6, [&] { hipLaunchKernelGGL(cal_store6, g, b, 0, 0, (uint32_t*)buf, n); });
    n = bytes;      run("cal_store1", n, n, [&] { hipLaunchKernelGGL(cal_store1, g, b, 0, 0, buf, n); });
    n = bytes / 16; run("cal_load16", n, n * 16, [&] { hipLaunchKernelGGL(cal_load16, g, b, 0, 0, (const uint4*)buf, n, sink); });
    n = bytes / 12; run("cal_load12", n, n * 12, [&] { hipLaunchKernelGGL(cal_load12, g, b, 0, 0, (const uint3*)buf, n, sink); });
    n = bytes / 8;  run("cal_load8", n, n * 8, [&] { hipLaunchKernelGGL(cal_load8, g, b, 0, 0, (const uint64_t*)buf, n, sink); });
    hipFree(buf);
    hipFree(sink);
    return 0;
}
