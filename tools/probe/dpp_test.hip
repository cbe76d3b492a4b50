#include "/root/repo/canonical-k-mer-hash-table_amd/csrc/kc_common.h"
#include <cstdio>
__global__ void k(const uint32_t* in, uint32_t* out) { out[threadIdx.x] = kc::wave_incl_sum(in[threadIdx.x]); }
int main() {
    uint32_t h[256], r[256]; for (int i = 0; i < 256; i++) h[i] = (i * 7919u) % 1000;
    uint32_t *d, *o; hipMalloc(&d, 1024); hipMalloc(&o, 1024); hipMemcpy(d, h, 1024, hipMemcpyHostToDevice);
    k<<<1, 256>>>(d, o); hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
    int bad = 0; for (int w = 0; w < 4; w++) { uint32_t acc = 0; for (int l = 0; l < 64; l++) { acc += h[w*64+l]; if (r[w*64+l] != acc) bad++; } }
    printf("dpp scan mismatches: %d\n", bad); return bad != 0;
}
