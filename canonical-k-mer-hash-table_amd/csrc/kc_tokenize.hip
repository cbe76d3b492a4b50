// kc_tokenize.hip -- bytes -> symbol stream, and the device read generator.
//
//   k_gather        device-resident source image -> TILE-aligned chunk stage
//   k_tile_summary  per 4 KiB tile: FASTA newline count + last header marker
//   k_tile_scan     one workgroup: stream offsets + header state entering each tile
//   k_emit          per tile: bytes -> symbol codes (0..3 base, 4 break); FASTA
//                   newlines are removed (they do not reset the window,
//                   parallel_parser.hpp:1432-1436), header bytes become breaks, and
//                   one break precedes every chunk (the k-mer factory is reset per
//                   chunk, parallel_parser.hpp:1310-1320)
//   k_synth         device twin of tools/kc_gen.c
//
// The tokenizer restates the per-byte loop of hash_kmers (parallel_parser.hpp:
// 1373-1465 FASTA, 1322-1372 plain) as a scan: the FASTA header state at a byte is
// the last of {'>' -> 1, '\n' -> 0, chunk start -> broken_header} at or before it.
#include "kc_common.h"
#include "kc_synth.h"

namespace kc {
// --------------------------------------------------------------------------------
// k_gather: copy chunks of a device-resident source image into the TILE-aligned stage
// (the device twin of the host's memcpy into pinned staging).
// --------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gather(const uint8_t* __restrict__ src, uint8_t* __restrict__ stage,
                                                const ChunkDesc* __restrict__ chunks) {
    const ChunkDesc c = chunks[blockIdx.y];
    const uint64_t per_block = 16 * 256 * 4;
    uint64_t base = (uint64_t)blockIdx.x * per_block;
    if (base >= c.len) return;
    const uint8_t* s = src + c.src_off;
    uint8_t* d = stage + c.stage_off;
    const bool aligned = ((c.src_off & 15) == 0);
    for (int r = 0; r < 4; r++) {
        uint64_t off = base + (uint64_t)r * 4096 + threadIdx.x * 16;
        if (off + 16 <= c.len) {
            if (aligned) {
                *reinterpret_cast<uint4*>(d + off) = *reinterpret_cast<const uint4*>(s + off);
            } else {
                uint4 v;
                uint8_t* pv = reinterpret_cast<uint8_t*>(&v);
#pragma unroll
                for (int j = 0; j < 16; j++) pv[j] = s[off + j];
                *reinterpret_cast<uint4*>(d + off) = v;
            }
        } else {
            for (uint64_t j = off; j < c.len && j < off + 16; j++) d[j] = s[j];
        }
    }
}

// chunk owning tile t (chunks sorted by stage_off, tiles contiguous)
DEV int find_chunk(const ChunkDesc* __restrict__ chunks, int n, uint64_t pos) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (chunks[mid].stage_off <= pos) lo = mid; else hi = mid - 1;
    }
    return lo;
}

DEV void load_tile_bytes(const uint8_t* __restrict__ p, uint32_t valid_here, uint8_t (&b)[16]) {
    if (valid_here >= 16) {
        uint4 v = *reinterpret_cast<const uint4*>(p);
        const uint8_t* pv = reinterpret_cast<const uint8_t*>(&v);
#pragma unroll
        for (int j = 0; j < 16; j++) b[j] = pv[j];
    } else {
#pragma unroll
        for (int j = 0; j < 16; j++) b[j] = (uint32_t)j < valid_here ? p[j] : 0;
    }
}

// --------------------------------------------------------------------------------
// k_tile_summary
// --------------------------------------------------------------------------------
__global__ __launch_bounds__(TILE_THREADS) void k_tile_summary(const uint8_t* __restrict__ stage,
                                                               const ChunkDesc* __restrict__ chunks, int n_chunks,
                                                               int fmt, TileInfo* __restrict__ tiles) {
    __shared__ uint32_t s_nl[TILE_THREADS / 64];
    __shared__ uint32_t s_mk[TILE_THREADS / 64];
    const uint64_t t = blockIdx.x;
    const uint64_t base = t * TILE;
    const int c = find_chunk(chunks, n_chunks, base);
    const ChunkDesc cd = chunks[c];
    const uint64_t rel = base - cd.stage_off;
    const uint32_t valid = (uint32_t)min((uint64_t)TILE, cd.len - rel);
    const int tid = threadIdx.x;
    const uint32_t my0 = tid * 16;
    const uint32_t vh = valid > my0 ? valid - my0 : 0;
    uint8_t b[16];
    load_tile_bytes(stage + base + my0, vh, b);
    uint32_t nl = 0, mk = 0;
    if (fmt == FMT_FASTA) {
#pragma unroll
        for (int j = 0; j < 16; j++) {
            if ((uint32_t)j < vh) {
                if (b[j] == '\n') { nl++; mk = 1; }
                else if (b[j] == '>') mk = 2;
            }
        }
    }
    // block reductions: sum of nl, last marker
    for (int d = 32; d >= 1; d >>= 1) nl += __shfl_xor(nl, d, 64);
    uint32_t tag = mk ? ((uint32_t)tid << 2) | mk : 0;
    for (int d = 32; d >= 1; d >>= 1) tag = max(tag, (uint32_t)__shfl_xor(tag, d, 64));
    if ((tid & 63) == 0) { s_nl[tid >> 6] = nl; s_mk[tid >> 6] = tag; }
    __syncthreads();
    if (tid == 0) {
        uint32_t tn = 0, tm = 0;
        for (int w = 0; w < TILE_THREADS / 64; w++) { tn += s_nl[w]; tm = max(tm, s_mk[w]); }
        TileInfo ti;
        ti.nl = tn;
        ti.valid = valid;
        ti.marker = (uint8_t)(tm & 3);
        ti.first = rel == 0;
        ti.bh = (uint8_t)cd.bh;
        ti.pad = 0;
        ti.pad2 = 0;
        tiles[t] = ti;
    }
}

// --------------------------------------------------------------------------------
// k_tile_scan: one 1024-thread workgroup over all tiles.
//   kept(t)  = valid - (FASTA ? nl : 0) + first   (one break symbol per chunk start)
//   hs_in(t) = first ? bh : hs_out(t-1);  hs_out = marker ? (marker == '>') : hs_in
// The header-state recurrence is a scan of "last defining tile" (a chunk start or a
// marker defines the state), composed left to right.
// --------------------------------------------------------------------------------
constexpr int SCAN_THREADS = 1024;
__global__ __launch_bounds__(SCAN_THREADS) void k_tile_scan(const TileInfo* __restrict__ tiles, uint64_t ntiles,
                                                           int fmt, TileOut* __restrict__ out,
                                                           DevCounters* __restrict__ ctr) {
    __shared__ unsigned long long s_sum[SCAN_THREADS];
    __shared__ uint32_t s_tr[SCAN_THREADS];
    const int tid = threadIdx.x;
    const uint64_t per = (ntiles + SCAN_THREADS - 1) / SCAN_THREADS;
    const uint64_t lo = min(ntiles, (uint64_t)tid * per), hi = min(ntiles, lo + per);
    unsigned long long sum = 0;
    uint32_t tr = 0;  // 0 identity, 1 const 0, 2 const 1
    for (uint64_t t = lo; t < hi; t++) {
        const TileInfo ti = tiles[t];
        sum += ti.valid - (fmt == FMT_FASTA ? ti.nl : 0) + ti.first;
        if (ti.marker) tr = ti.marker == 2 ? 2 : 1;
        else if (ti.first) tr = ti.bh ? 2 : 1;
    }
    s_sum[tid] = sum;
    s_tr[tid] = tr;
    __syncthreads();
    // Hillis-Steele inclusive scans in LDS
    for (int d = 1; d < SCAN_THREADS; d <<= 1) {
        unsigned long long vs = tid >= d ? s_sum[tid - d] : 0;
        uint32_t vt = tid >= d ? s_tr[tid - d] : 0;
        __syncthreads();
        s_sum[tid] += vs;
        if (s_tr[tid] == 0) s_tr[tid] = vt;
        __syncthreads();
    }
    unsigned long long run = tid ? s_sum[tid - 1] : 0;
    uint32_t st = tid ? (s_tr[tid - 1] == 2 ? 1u : 0u) : 0u;
    for (uint64_t t = lo; t < hi; t++) {
        const TileInfo ti = tiles[t];
        TileOut to;
        to.out_off = run;
        uint32_t hin = ti.first ? ti.bh : st;
        to.hs_in = fmt == FMT_FASTA ? hin : 0;
        to.pad = 0;
        out[t] = to;
        st = ti.marker ? (ti.marker == 2 ? 1u : 0u) : hin;
        run += ti.valid - (fmt == FMT_FASTA ? ti.nl : 0) + ti.first;
    }
    if (tid == SCAN_THREADS - 1) ctr->stream_len = s_sum[SCAN_THREADS - 1];
}

// --------------------------------------------------------------------------------
// k_emit: bytes -> symbol codes
// --------------------------------------------------------------------------------
__global__ __launch_bounds__(TILE_THREADS) void k_emit(const uint8_t* __restrict__ stage,
                                                       const TileInfo* __restrict__ tiles,
                                                       const TileOut* __restrict__ touts, int fmt,
                                                       uint64_t* __restrict__ pk, uint32_t* __restrict__ bk) {
    __shared__ uint8_t s_codes[TILE + 16];
    __shared__ uint32_t s_wsum[TILE_THREADS / 64];
    __shared__ uint32_t s_wmk[TILE_THREADS / 64];
    const uint64_t t = blockIdx.x;
    const TileInfo ti = tiles[t];
    const TileOut to = touts[t];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t my0 = tid * 16;
    const uint32_t vh = ti.valid > my0 ? ti.valid - my0 : 0;
    uint8_t b[16];
    load_tile_bytes(stage + t * TILE + my0, vh, b);

    uint32_t state = 0;
    if (fmt == FMT_FASTA) {
        // header state entering this thread: last marker of the lower threads, else hs_in
        uint32_t mk = 0;
#pragma unroll
        for (int j = 0; j < 16; j++)
            if ((uint32_t)j < vh) {
                if (b[j] == '\n') mk = 1;
                else if (b[j] == '>') mk = 2;
            }
        uint32_t incl = wave_incl_last(mk);
        if (lane == 63) s_wmk[wid] = incl;
        __syncthreads();
        uint32_t excl = __shfl_up(incl, 1, 64);
        if (lane == 0) excl = 0;
        if (excl == 0) {
            for (int w = wid - 1; w >= 0; w--)
                if (s_wmk[w]) { excl = s_wmk[w]; break; }
        }
        state = excl ? (excl == 2 ? 1u : 0u) : to.hs_in;
    }

    uint8_t codes[16];
    uint32_t kept = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        codes[j] = 0xff;
        if ((uint32_t)j < vh) {
            const uint8_t ch = b[j];
            if (fmt == FMT_FASTA) {
                if (ch == '\n') { state = 0; continue; }
                if (ch == '>') state = 1;
                codes[j] = state ? SYM_BREAK : char_code(ch);
            } else {
                codes[j] = char_code(ch);
            }
            kept++;
        }
    }
    uint32_t incl = wave_incl_sum(kept);
    if (lane == 63) s_wsum[wid] = incl;
    __syncthreads();
    // a chunk's first tile starts with the chunk-separating break
    uint32_t pos = incl - kept + ti.first;
    uint32_t total = ti.first;
    for (int w = 0; w < TILE_THREADS / 64; w++) {
        if (w < wid) pos += s_wsum[w];
        total += s_wsum[w];
    }
    if (ti.first && tid == 0) s_codes[0] = SYM_BREAK;
#pragma unroll
    for (int j = 0; j < 16; j++)
        if (codes[j] != 0xff) s_codes[pos++] = codes[j];
    __syncthreads();
    if (total == 0) return;
    // pack: 32 symbols per word, symbol j of word w at bits 62-2j (codes) / 31-j (breaks);
    // words shared with the neighbouring tiles are OR-ed into the zeroed buffers
    const uint64_t g0 = to.out_off;
    const uint64_t w_lo = g0 >> 5, w_hi = (g0 + total - 1) >> 5;
    for (uint64_t w = w_lo + tid; w <= w_hi; w += TILE_THREADS) {
        const int64_t l0 = (int64_t)(w << 5) - (int64_t)g0;
        uint64_t pv = 0;
        uint32_t bv = 0;
#pragma unroll 8
        for (int j = 0; j < 32; j++) {
            const int64_t l = l0 + j;
            if (l >= 0 && l < (int64_t)total) {
                const uint8_t c = s_codes[l];
                if (c > 3) bv |= 1u << (31 - j);
                else pv |= (uint64_t)c << (62 - 2 * j);
            }
        }
        if (l0 >= 0 && l0 + 32 <= (int64_t)total) {
            pk[w] = pv;
            bk[w] = bv;
        } else {
            if (pv) atomicOr((unsigned long long*)(pk + w), (unsigned long long)pv);
            if (bv) atomicOr(bk + w, bv);
        }
    }
}


// --------------------------------------------------------------------------------
// k_synth: device twin of tools/kc_gen.c (one thread per read)
// --------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_synth(uint8_t* __restrict__ dst, uint64_t first, uint64_t n,
                                               kc_synth_params p, uint64_t base_off) {
    const uint64_t r = first + (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= first + n) return;
    const uint64_t e_th = kcs_thresh(p.err_rate), n_th = kcs_thresh(p.n_rate);
    uint8_t* o = dst + (kcs_record_offset(&p, r) - base_off);
    // header ">r<i>\n"
    const int nd = kcs_digits(r);
    o[0] = '>';
    o[1] = 'r';
    uint64_t v = r;
    for (int d = nd - 1; d >= 0; d--) { o[2 + d] = (uint8_t)('0' + v % 10); v /= 10; }
    o[2 + nd] = '\n';
    o += 3 + nd;
    const uint64_t st = kcs_read_start(&p, r);
    const int rc = kcs_read_rc(&p, r);
    const char sy[5] = {'A', 'C', 'G', 'T', 'N'};
    uint32_t col = 0;
    for (uint32_t j = 0; j < p.read_len; j++) {
        *o++ = (uint8_t)sy[kcs_read_base(&p, r, j, st, rc, e_th, n_th)];
        if (p.wrap && ++col == p.wrap && j + 1 < p.read_len) { *o++ = '\n'; col = 0; }
    }
    *o = '\n';
}

// ================================================================================
// launchers
// ================================================================================

// ================================================================================
// launchers
// ================================================================================
hipError_t launch_gather(const uint8_t* src, uint8_t* stage, const ChunkDesc* d_chunks, int n_chunks,
                         const ChunkDesc* h_chunks, hipStream_t s) {
    uint64_t maxlen = 0;
    for (int i = 0; i < n_chunks; i++) maxlen = h_chunks[i].len > maxlen ? h_chunks[i].len : maxlen;
    const uint64_t per_block = 16 * 256 * 4;
    dim3 grid((unsigned)((maxlen + per_block - 1) / per_block), (unsigned)n_chunks);
    hipLaunchKernelGGL(k_gather, grid, dim3(256), 0, s, src, stage, d_chunks);
    return hipGetLastError();
}

hipError_t launch_tokenize(const uint8_t* stage, uint64_t ntiles, const ChunkDesc* d_chunks, int n_chunks, int fmt,
                           TileInfo* tiles, TileOut* touts, PackedView sv, uint64_t sym_bound, DevCounters* ctr,
                           hipStream_t s) {
    const uint64_t words = sym_bound / 32 + 2;
    hipError_t e;
    if ((e = hipMemsetAsync(sv.pk, 0, words * 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(sv.bk, 0, words * 4, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_tile_summary, dim3((unsigned)ntiles), dim3(TILE_THREADS), 0, s, stage, d_chunks, n_chunks,
                       fmt, tiles);
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(SCAN_THREADS), 0, s, tiles, ntiles, fmt, touts, ctr);
    hipLaunchKernelGGL(k_emit, dim3((unsigned)ntiles), dim3(TILE_THREADS), 0, s, stage, tiles, touts, fmt, sv.pk, sv.bk);
    return hipGetLastError();
}

hipError_t launch_synth(uint8_t* dst, uint64_t first_read, uint64_t n_reads, uint64_t seed, uint64_t genome_len,
                        uint32_t read_len, uint32_t wrap, double err_rate, double n_rate, hipStream_t s) {
    kc_synth_params p;
    p.seed = seed;
    p.genome_len = genome_len;
    p.n_reads = first_read + n_reads;
    p.read_len = read_len;
    p.wrap = wrap;
    p.err_rate = err_rate;
    p.n_rate = n_rate;
    const uint64_t base = kcs_record_offset(&p, first_read);
    const unsigned grid = (unsigned)((n_reads + 255) / 256);
    if (grid) hipLaunchKernelGGL(k_synth, dim3(grid), dim3(256), 0, s, dst, first_read, n_reads, p, base);
    return hipGetLastError();
}

}  // namespace kc
