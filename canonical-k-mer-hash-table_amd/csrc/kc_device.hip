// kc_device.hip -- MI355X (gfx950) kernels of the canonical k-mer counting path.
//
// Pipeline per staged batch (the reference's per-chunk worker loop
// parallel_parser.hpp:1373-1465 / 1322-1372 re-designed as data-parallel passes):
//   k_gather        device-resident source image -> TILE-aligned chunk stage
//   k_tile_summary  per 4 KiB tile: FASTA newline count + last header marker
//   k_tile_scan     one workgroup: stream offsets + header state entering each tile
//   k_emit          per tile: bytes -> symbol stream (0..3 base, 4 break), FASTA
//                   newlines removed (they do not reset, parallel_parser.hpp:1432-1436),
//                   header bytes -> break, one break in front of every chunk
//   k_count<W,MODE> per thread RUN consecutive symbols: roll 2-bit forward and
//                   reverse-complement words (kmer_factory.cpp:172-239), canonical
//                   = min, then insert into the open-address table
//                   (replaces process_kmer_MT, kmer_hash_table.cpp:2207-2567), or the
//                   double Bloom filter pass 1 (double_bloomfilter.hpp:371-413), or
//                   the pass-2 gate (parallel_parser.hpp:2436-2453)
//   k_dump<W>       table -> (key words, T(c)) records with T(c) >= a
//                   (replaces write_kmers_on_disk_separately_even_faster,
//                   kmer_hash_table.cpp:4318-4524, and write_kmers 2013-2050)
//
// Table: 128-byte buckets, keys [S][W] u64 then counts [S] u64, S = 16/(W+1).
// Word 0 of a key is the most significant and always has spare top bits (W = k/32+1),
// so a stored word 0 carries the OCC tag bit and 0 is EMPTY (a zeroed table is
// empty).  W == 1 keys are claimed by one 64-bit CAS.  W > 1 keys are
// claimed by a CAS of word 0, the other words are written with agent-scope atomic
// stores, drained, and published by adding READY|1 to the count word; readers
// that match word 0 wait (retrying the slot) until READY is visible.
#include "kc_internal.h"
#include "kc_synth.h"

namespace kc {

#define DEV __device__ __forceinline__

// --------------------------------------------------------------------------------
// small helpers
// --------------------------------------------------------------------------------
DEV uint8_t char_code(uint8_t c) {  // functions_strings.cpp:56-70
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return SYM_BREAK;
    }
}

DEV uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}

template <int W>
DEV uint64_t key_hash(const uint64_t (&key)[W]) {
    uint64_t h = fmix64(key[W - 1] ^ 0x243f6a8885a308d3ULL);
#pragma unroll
    for (int i = W - 2; i >= 0; i--) h = fmix64(h ^ key[i]);
    return h;
}

// wave-level inclusive scans (64 lanes)
DEV uint32_t wave_incl_sum(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}
DEV uint32_t wave_incl_last(uint32_t v) {  // last non-zero value up to this lane
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t o = __shfl_up(v, d, 64);
        if (lane >= d && v == 0) v = o;
    }
    return v;
}

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
                                                       uint8_t* __restrict__ sym) {
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
    uint32_t pos = incl - kept;
    uint32_t total = 0;
    for (int w = 0; w < TILE_THREADS / 64; w++) {
        if (w < wid) pos += s_wsum[w];
        total += s_wsum[w];
    }
#pragma unroll
    for (int j = 0; j < 16; j++)
        if (codes[j] != 0xff) s_codes[pos++] = codes[j];
    __syncthreads();
    uint8_t* dst = sym + to.out_off;
    if (ti.first) {
        if (tid == 0) dst[0] = SYM_BREAK;
        dst += 1;
    }
    for (uint32_t i = tid; i < total; i += TILE_THREADS) dst[i] = s_codes[i];
}

// --------------------------------------------------------------------------------
// XXH64 of one 8-byte value (xxhash.h:3368-3509 / doc/xxhash_spec.md:191-334)
// --------------------------------------------------------------------------------
__constant__ uint64_t c_bf_seeds[MAX_NH] = {2411, 3253, 1061, 1129, 2269, 7309, 3491, 8237, 6359, 8779};

DEV uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
DEV uint64_t xxh64_u64(uint64_t v, uint64_t seed) {
    const uint64_t P1 = 0x9E3779B185EBCA87ULL, P2 = 0xC2B2AE3D27D4EB4FULL, P3 = 0x165667B19E3779F9ULL,
                   P4 = 0x85EBCA77C2B2AE63ULL, P5 = 0x27D4EB2F165667C5ULL;
    uint64_t h = seed + P5 + 8;
    uint64_t k1 = rotl64(v * P2, 31) * P1;
    h ^= k1;
    h = rotl64(h, 27) * P1 + P4;
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

// --------------------------------------------------------------------------------
// Table insert (one canonical key)
// --------------------------------------------------------------------------------
DEV uint64_t atomic_load_agent(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV void atomic_store_agent(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int W>
DEV bool table_insert(const TableView& tv, const uint64_t (&key)[W]) {
    constexpr int S = BUCKET_WORDS / (W + 1);
    const uint64_t h = key_hash<W>(key);
    uint64_t bkt = __umul64hi(h, tv.nbuckets);
    for (uint64_t probe = 0; probe < tv.nbuckets; probe++) {
        uint64_t* b = tv.buckets + bkt * BUCKET_WORDS;
        uint64_t w0[S];
        if constexpr (W == 1) {
            const uint4* b4 = reinterpret_cast<const uint4*>(b);
#pragma unroll
            for (int q = 0; q < S / 2; q++) {
                uint4 v = b4[q];
                w0[2 * q] = ((uint64_t)v.y << 32) | v.x;
                w0[2 * q + 1] = ((uint64_t)v.w << 32) | v.z;
            }
        } else {
#pragma unroll
            for (int s = 0; s < S; s++) w0[s] = b[s * W];
        }
        int s = 0;
        while (s < S) {
            uint64_t* kp = b + s * W;
            uint64_t* cp = b + S * W + s;
            uint64_t v0 = w0[s];
            if (v0 == EMPTY) {
                uint64_t old = atomicCAS((unsigned long long*)kp, (unsigned long long)EMPTY,
                                         (unsigned long long)(key[0] | OCC));
                if (old == EMPTY) {
                    if constexpr (W == 1) {
                        atomicAdd((unsigned long long*)cp, 1ULL);
                    } else {
#pragma unroll
                        for (int i = 1; i < W; i++) atomic_store_agent(kp + i, key[i]);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the word stores, then publish
                        atomicAdd((unsigned long long*)cp, (unsigned long long)(READY + 1));
                    }
                    return true;
                }
                v0 = old;
                w0[s] = old;
            }
            if (v0 == (key[0] | OCC)) {
                if constexpr (W == 1) {
                    atomicAdd((unsigned long long*)cp, 1ULL);
                    return true;
                } else {
                    const uint64_t c = atomic_load_agent(cp);
                    if (!(c & READY)) continue;  // claimed but not yet published: retry this slot
                    asm volatile("" ::: "memory");
                    bool eq = true;
#pragma unroll
                    for (int i = 1; i < W; i++) eq &= atomic_load_agent(kp + i) == key[i];
                    if (eq) {
                        atomicAdd((unsigned long long*)cp, 1ULL);
                        return true;
                    }
                }
            }
            s++;
        }
        bkt = bkt + 1 == tv.nbuckets ? 0 : bkt + 1;
    }
    return false;
}

// --------------------------------------------------------------------------------
// Bloom filter (double filter in one interleaved bit array)
// --------------------------------------------------------------------------------
struct BloomLocal {
    uint32_t new_first, new_second, failed;
};

// insertion_process (double_bloomfilter.hpp:371-413); every "set" is an atomicOr and
// counts as ours only if it flipped the bit (MyAtomicBitArrayFT::set, mybitarray.hpp:87-125)
DEV void bloom_insert(const BloomView& bf, uint64_t root, BloomLocal& loc) {
    uint64_t widx[MAX_NH];
    uint32_t bpos[MAX_NH];
    uint32_t view[MAX_NH];
    int s1 = 0, s2 = 0;
#pragma unroll
    for (int j = 0; j < MAX_NH; j++) {
        if (j < bf.nh) {
            const uint64_t hv = xxh64_u64(root, c_bf_seeds[j]) & bf.mask;
            const uint64_t bit = 2 * hv;
            widx[j] = bit >> 5;
            bpos[j] = (uint32_t)(bit & 31);
            view[j] = bf.bits[widx[j]];
        }
    }
#pragma unroll
    for (int j = 0; j < MAX_NH; j++)
        if (j < bf.nh) {
            s1 += (view[j] >> bpos[j]) & 1;
            s2 += (view[j] >> (bpos[j] + 1)) & 1;
        }
    if (s2 == bf.nh) return;
    bool to_second;
    if (s1 == bf.nh) {
        to_second = true;
    } else {
        int mine = 0;
#pragma unroll
        for (int j = 0; j < MAX_NH; j++)
            if (j < bf.nh) {
                const uint32_t m = 1u << bpos[j];
                if (!(view[j] & m)) {
                    const uint32_t old = atomicOr(bf.bits + widx[j], m);
                    if (!(old & m)) mine++;
                    view[j] = old | m;
                }
            }
        if (mine == bf.nh - s1) { loc.new_first++; to_second = false; }
        else { loc.failed++; to_second = true; }
    }
    if (to_second) {
        int mine = 0;
#pragma unroll
        for (int j = 0; j < MAX_NH; j++)
            if (j < bf.nh) {
                const uint32_t m = 2u << bpos[j];
                if (!(view[j] & m)) {
                    const uint32_t old = atomicOr(bf.bits + widx[j], m);
                    if (!(old & m)) mine++;
                }
            }
        if (mine == bf.nh - s2) loc.new_second++;
    }
}

// pass-2 gate: all of the first trunc(hf) filter-2 bits set (parallel_parser.hpp:2436-2441)
DEV bool bloom_gate(const BloomView& bf, uint64_t root) {
    bool all = true;
#pragma unroll
    for (int j = 0; j < MAX_NH; j++)
        if (j < bf.nh_gate) {
            const uint64_t bit = 2 * (xxh64_u64(root, c_bf_seeds[j]) & bf.mask) + 1;
            all &= (bf.bits[bit >> 5] >> (bit & 31)) & 1;
        }
    return all;
}

// --------------------------------------------------------------------------------
// k_count<W, MODE>
// --------------------------------------------------------------------------------
constexpr uint64_t M54 = (1ULL << 54) - 1;
constexpr uint64_t INV5_54 = 0xCCCCCCCCCCCCDULL;  // 5 * INV5_54 == 1 (mod 2^54)

template <int W, int MODE>
__global__ __launch_bounds__(COUNT_THREADS) void k_count(const uint8_t* __restrict__ sym, int k, TableView tv,
                                                         BloomView bf, DevCounters* __restrict__ ctr,
                                                         uint64_t pow5_k, uint64_t pow5_km1) {
    __shared__ unsigned long long s_red[4][COUNT_THREADS / 64];
    const uint64_t M = ctr->stream_len;
    const uint64_t gid = (uint64_t)blockIdx.x * COUNT_THREADS + threadIdx.x;
    const uint64_t p0 = gid * RUN;
    uint32_t n_win = 0, n_ins = 0, n_fail_tab = 0;
    BloomLocal bl = {0, 0, 0};
    if (p0 < M) {
        const uint64_t pstart = p0 >= (uint64_t)(k - 1) ? p0 - (k - 1) : 0;
        const uint64_t pend = min(p0 + RUN, M);
        const int top = 2 * k - 64 * (W - 1);                 // bits used in word 0 (0..62)
        const uint64_t topmask = top >= 64 ? ~0ULL : ((1ULL << top) - 1);
        const int rc_word = W - 1 - (2 * k - 2) / 64;
        const int rc_bit = (2 * k - 2) % 64;
        const int out_word = W - 1 - (2 * k - 2) / 64;   // word holding the oldest character
        uint64_t fwd[W], rc[W];
#pragma unroll
        for (int i = 0; i < W; i++) { fwd[i] = 0; rc[i] = 0; }
        int fill = 0;
        uint64_t F = 0, B = 0, p5 = 1;  // Rabin-Karp mod 2^54 (hash_functions.cpp:102-192)
        for (uint64_t p = pstart; p < pend; p++) {
            const uint8_t c = sym[p];
            if (c > 3) {
                fill = 0;
#pragma unroll
                for (int i = 0; i < W; i++) { fwd[i] = 0; rc[i] = 0; }
                if constexpr (MODE != 0) { F = 0; B = 0; p5 = 1; }
                continue;
            }
            if constexpr (MODE != 0) {
                if (fill < k) {
                    F = (F * 5 + c) & M54;
                    B = (B + (uint64_t)(3 - c) * p5) & M54;
                    p5 = (p5 * 5) & M54;
                } else {
                    const uint64_t out = (fwd[out_word] >> rc_bit) & 3;
                    F = (F * 5 + c - pow5_k * out) & M54;
                    B = (((B - (3 - out)) & M54) * INV5_54 + (uint64_t)(3 - c) * pow5_km1) & M54;
                }
            }
#pragma unroll
            for (int i = 0; i < W - 1; i++) fwd[i] = (fwd[i] << 2) | (fwd[i + 1] >> 62);
            fwd[W - 1] = (fwd[W - 1] << 2) | c;
            fwd[0] &= topmask;
#pragma unroll
            for (int i = W - 1; i >= 1; i--) rc[i] = (rc[i] >> 2) | (rc[i - 1] << 62);
            rc[0] >>= 2;
#pragma unroll
            for (int i = 0; i < W; i++)
                if (i == rc_word) rc[i] |= (uint64_t)(3 - c) << rc_bit;
            if (fill < k) fill++;
            if (fill == k && p >= p0) {
                n_win++;
                if constexpr (MODE == 1) {
                    bloom_insert(bf, F < B ? F : B, bl);
                } else {
                    if constexpr (MODE == 2) {
                        if (!bloom_gate(bf, F < B ? F : B)) continue;
                    }
                    bool fwd_le = true;
#pragma unroll
                    for (int i = W - 1; i >= 0; i--)
                        if (fwd[i] != rc[i]) fwd_le = fwd[i] < rc[i];
                    uint64_t key[W];
#pragma unroll
                    for (int i = 0; i < W; i++) key[i] = fwd_le ? fwd[i] : rc[i];
                    n_ins++;
                    if (!table_insert<W>(tv, key)) n_fail_tab++;
                }
            }
        }
    }
    // block reduction -> one sharded atomic per counter
    unsigned long long v[4] = {n_win, n_ins, n_fail_tab, 0};
    if constexpr (MODE == 1) { v[1] = bl.new_first; v[2] = bl.new_second; v[3] = bl.failed; }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        unsigned long long x = v[q];
        for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
        if (lane == 0) s_red[q][wid] = x;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        unsigned long long x = 0;
        for (int w = 0; w < COUNT_THREADS / 64; w++) x += s_red[threadIdx.x][w];
        if (x) {
            unsigned long long* dst;
            if constexpr (MODE == 1) {
                dst = threadIdx.x == 0 ? &ctr->bf_windows
                    : threadIdx.x == 1 ? &ctr->new_in_first
                    : threadIdx.x == 2 ? &ctr->new_in_second : &ctr->failed_in_first;
            } else {
                dst = threadIdx.x == 0 ? &ctr->windows : threadIdx.x == 1 ? &ctr->inserted : &ctr->overflow;
            }
            atomicAdd(dst, x);
        }
    }
}

// --------------------------------------------------------------------------------
// k_dump<W>: occupied slots with T(c) >= a -> records {W key words, T(c)}
// count_mode 0: c mod 65536 (-m 0); else min(c, 16383)
// --------------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(256) void k_dump(TableView tv, int count_mode, uint64_t min_abundance,
                                              uint64_t* __restrict__ out, DevCounters* __restrict__ ctr) {
    constexpr int S = BUCKET_WORDS / (W + 1);
    const uint64_t bkt = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t occ = 0, nout = 0;
    uint64_t tv_c[S];
    bool emit[S];
    const uint64_t* b = tv.buckets + bkt * BUCKET_WORDS;
#pragma unroll
    for (int s = 0; s < S; s++) {
        emit[s] = false;
        tv_c[s] = 0;
        if (bkt < tv.nbuckets && b[s * W] != EMPTY) {
            occ++;
            const uint64_t c = b[S * W + s] & CNT_MASK;
            const uint64_t t = count_mode == 0 ? (c & 0xFFFF) : (c < 16383 ? c : 16383);
            if (t >= min_abundance) { emit[s] = true; tv_c[s] = t; nout++; }
        }
    }
    // wave-aggregated output allocation
    const int lane = threadIdx.x & 63;
    uint32_t incl = wave_incl_sum(nout);
    uint32_t wtot = __shfl(incl, 63, 64);
    unsigned long long base = 0;
    if (lane == 63 && wtot) base = atomicAdd(&ctr->dump_n, (unsigned long long)wtot);
    base = __shfl(base, 63, 64);
    uint64_t idx = base + incl - nout;
#pragma unroll
    for (int s = 0; s < S; s++)
        if (out && emit[s]) {
            uint64_t* o = out + idx * (W + 1);
#pragma unroll
            for (int i = 0; i < W; i++) o[i] = b[s * W + i] & (i == 0 ? ~OCC : ~0ULL);
            o[W] = tv_c[s];
            idx++;
        }
    uint32_t occ_w = occ;
    for (int d = 32; d >= 1; d >>= 1) occ_w += __shfl_xor(occ_w, d, 64);
    if (lane == 0 && occ_w) atomicAdd(&ctr->occupied, (unsigned long long)occ_w);
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
                           TileInfo* tiles, TileOut* touts, uint8_t* sym, uint64_t sym_cap, DevCounters* ctr,
                           hipStream_t s) {
    (void)sym_cap;
    hipLaunchKernelGGL(k_tile_summary, dim3((unsigned)ntiles), dim3(TILE_THREADS), 0, s, stage, d_chunks, n_chunks,
                       fmt, tiles);
    hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(SCAN_THREADS), 0, s, tiles, ntiles, fmt, touts, ctr);
    hipLaunchKernelGGL(k_emit, dim3((unsigned)ntiles), dim3(TILE_THREADS), 0, s, stage, tiles, touts, fmt, sym);
    return hipGetLastError();
}

static uint64_t pow5_mod54(int e) {
    uint64_t r = 1;
    for (int i = 0; i < e; i++) r = (r * 5) & M54;
    return r;
}

template <int W>
static hipError_t launch_count_w(const uint8_t* sym, uint64_t sym_bound, int k, int mode, TableView t, BloomView bf,
                                 DevCounters* ctr, hipStream_t s) {
    const uint64_t threads = (sym_bound + RUN - 1) / RUN;
    const unsigned grid = (unsigned)((threads + COUNT_THREADS - 1) / COUNT_THREADS);
    const uint64_t pk = pow5_mod54(k), pkm1 = pow5_mod54(k - 1);
    if (grid == 0) return hipSuccess;
    if (mode == 0)
        hipLaunchKernelGGL((k_count<W, 0>), dim3(grid), dim3(COUNT_THREADS), 0, s, sym, k, t, bf, ctr, pk, pkm1);
    else if (mode == 1)
        hipLaunchKernelGGL((k_count<W, 1>), dim3(grid), dim3(COUNT_THREADS), 0, s, sym, k, t, bf, ctr, pk, pkm1);
    else
        hipLaunchKernelGGL((k_count<W, 2>), dim3(grid), dim3(COUNT_THREADS), 0, s, sym, k, t, bf, ctr, pk, pkm1);
    return hipGetLastError();
}

hipError_t launch_count(const uint8_t* sym, uint64_t sym_bound, int k, int mode, TableView t, BloomView bf,
                        DevCounters* ctr, hipStream_t s) {
    switch (words_for_k(k)) {
    case 1: return launch_count_w<1>(sym, sym_bound, k, mode, t, bf, ctr, s);
    case 2: return launch_count_w<2>(sym, sym_bound, k, mode, t, bf, ctr, s);
    case 3: return launch_count_w<3>(sym, sym_bound, k, mode, t, bf, ctr, s);
    case 4: return launch_count_w<4>(sym, sym_bound, k, mode, t, bf, ctr, s);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_dump(TableView t, int count_mode, uint64_t min_abundance, uint64_t* out, DevCounters* ctr,
                       hipStream_t s) {
    const unsigned grid = (unsigned)((t.nbuckets + 255) / 256);
    switch (t.W) {
    case 1: hipLaunchKernelGGL(k_dump<1>, dim3(grid), dim3(256), 0, s, t, count_mode, min_abundance, out, ctr); break;
    case 2: hipLaunchKernelGGL(k_dump<2>, dim3(grid), dim3(256), 0, s, t, count_mode, min_abundance, out, ctr); break;
    case 3: hipLaunchKernelGGL(k_dump<3>, dim3(grid), dim3(256), 0, s, t, count_mode, min_abundance, out, ctr); break;
    case 4: hipLaunchKernelGGL(k_dump<4>, dim3(grid), dim3(256), 0, s, t, count_mode, min_abundance, out, ctr); break;
    default: return hipErrorInvalidValue;
    }
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
