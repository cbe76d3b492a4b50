// kc_tokenize.hip -- bytes -> symbol stream, and the device read generator.
//
//   k_tile_summary  per 4 KiB tile: FASTA/FASTQ newline count + last FASTA header marker
//   k_tscan_*       two-level scan: stream offsets + header state entering each tile
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
//
// FASTQ (an extension: the reference rejects it, parallel_parser.hpp:1216-1225): chunks
// hold whole 4-line records (kc_plan_chunks), so the line of a byte is (newlines
// before it in the batch) mod 4; only line 1 (the sequence) yields symbols, every
// other byte and every newline is a break -- the counts equal those of the plain-text
// file of the sequence lines.  The newline count rides in bits 40.. of the tile scan's
// symbol sum (only its value mod 4 is used; a batch holds < 2^40 symbols).
#include <cstdlib>

#include "kc_common.h"
#include "kc_synth.h"

namespace kc {
// ---- 16 source bytes per thread, as four little-endian words ----------------------
// The tile's bytes are read straight from the source (device image or host stage) at
// the chunk's offset, which has any alignment: five aligned dwords are funnel-shifted.
// The fast path needs 3 readable bytes past the 16 (still inside the chunk), so the
// last few bytes of a chunk take the byte path and nothing is read past a chunk.
// Two phases, so that a workgroup's loads for several tiles are all issued before the
// first is used (a funnel shift right after its loads makes the compiler wait for them):
// load16_issue loads the five dwords of the fast path (a lane whose 16 bytes are not
// followed by 3 readable ones issues nothing), load16_finish shifts them, or reads the
// bytes of the rare short case.
DEV bool load16_fast(uint32_t vh) { return vh >= 19; }
DEV void load16_issue(const uint8_t* __restrict__ p, uint32_t (&x)[5]) {
    // (p minus its misalignment, not the masked integer, so the compiler still sees a global
    // pointer: a flat load also counts against lgkmcnt, and the next scalar load's wait stalls on it)
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p - (reinterpret_cast<uintptr_t>(p) & 3));
#pragma unroll
    for (int i = 0; i < 5; i++) x[i] = q[i];
}
DEV void load16_finish(const uint8_t* __restrict__ p, uint32_t vh, const uint32_t (&x)[5], uint32_t (&w)[4]) {
    if (load16_fast(vh)) {
        const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
#pragma unroll
        for (int i = 0; i < 4; i++) w[i] = __builtin_amdgcn_alignbyte(x[i + 1], x[i], sh);
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint32_t v = 0;
#pragma unroll
            for (int j = 0; j < 4; j++)
                if ((uint32_t)(4 * i + j) < vh) v |= (uint32_t)p[4 * i + j] << (8 * j);
            w[i] = v;
        }
    }
}

// ---- SWAR byte classification ------------------------------------------------------
DEV uint32_t zero_bytes(uint32_t v) {  // 0x80 in exactly the bytes of v that are 0
    const uint32_t t = (v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    return ~(t | v | 0x7F7F7F7Fu);
}
DEV uint32_t flags4(uint32_t z) { return ((z >> 7) * 0x10204080u) >> 28; }  // bit i = byte i's 0x80
DEV uint32_t eq_mask16(const uint32_t (&w)[4], uint32_t pat) {  // bit j: byte j == pattern byte
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) m |= flags4(zero_bytes(w[i] ^ pat)) << (4 * i);
    return m;
}

// --------------------------------------------------------------------------------
// k_tile_map: the chunk of every tile (a chunk's tiles are the TILE-aligned slots it
// occupies in the stage), parked in tiles[t].nl for k_tile_summary, which replaces a
// per-tile binary search over the chunk table (dependent loads, ~8 per tile) by one load
// --------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_tile_map(const ChunkDesc* __restrict__ chunks, TileInfo* __restrict__ tiles) {
    const ChunkDesc cd = chunks[blockIdx.x];
    const uint64_t t0 = cd.stage_off / TILE, t1 = (cd.stage_off + cd.len + TILE - 1) / TILE;
    for (uint64_t t = t0 + threadIdx.x; t < t1; t += 256) tiles[t].nl = blockIdx.x;
}

// --------------------------------------------------------------------------------
// k_tile_summary_m<TPB>: per 4 KiB tile the FASTA/FASTQ newline count and the last FASTA header
// marker, for TPB consecutive tiles per workgroup,
// every thread's TPB loads (tile map -> chunk descriptor -> 16 bytes of each tile) issued
// before any is used: one 4 KiB tile per workgroup left a chain of three dependent loads per
// 16 bytes in flight, the summary ran at ~3.5 TB/s of its 1.6 GB (C2)
template <int TPB>
__global__ __launch_bounds__(TILE_THREADS) void k_tile_summary_m(const uint8_t* __restrict__ src,
                                                                 const ChunkDesc* __restrict__ chunks, uint64_t ntiles,
                                                                 int fmt, TileInfo* __restrict__ tiles) {
    __shared__ uint32_t s_nl[TPB][TILE_THREADS / 64];
    __shared__ uint32_t s_mk[TPB][TILE_THREADS / 64];
    const int tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * TPB;
    int ci[TPB];
#pragma unroll
    for (int j = 0; j < TPB; j++) ci[j] = t0 + j < ntiles ? (int)tiles[t0 + j].nl : 0;  // k_tile_map
    ChunkDesc cd[TPB];
#pragma unroll
    for (int j = 0; j < TPB; j++) cd[j] = chunks[ci[j]];
    uint32_t w[TPB][4], vh[TPB], valid[TPB], avail[TPB], x[TPB][5];
    uint64_t rel[TPB];
    const uint32_t my0 = tid * 16;
#pragma unroll
    for (int j = 0; j < TPB; j++) {  // every tile's dword loads first (load16_issue)
        rel[j] = (t0 + j) * TILE - cd[j].stage_off;
        const bool in = t0 + j < ntiles;
        valid[j] = in ? (uint32_t)min((uint64_t)TILE, cd[j].len - rel[j]) : 0;
        avail[j] = in ? (uint32_t)min((uint64_t)TILE + 64, cd[j].len - rel[j]) : 0;
        vh[j] = valid[j] > my0 ? valid[j] - my0 : 0;
        if (fmt != FMT_PLAIN && vh[j] && load16_fast(avail[j] - my0))
            load16_issue(src + cd[j].src_off + rel[j] + my0, x[j]);
    }
#pragma unroll
    for (int j = 0; j < TPB; j++) {
        w[j][0] = w[j][1] = w[j][2] = w[j][3] = 0;
        if (fmt != FMT_PLAIN && vh[j]) load16_finish(src + cd[j].src_off + rel[j] + my0, avail[j] - my0, x[j], w[j]);
    }
#pragma unroll
    for (int j = 0; j < TPB; j++) {
        uint32_t nl = 0, mk = 0;
        if (fmt != FMT_PLAIN && vh[j]) {
            const uint32_t vmask = vh[j] >= 16 ? 0xFFFFu : ((1u << vh[j]) - 1);
            const uint32_t nlm = eq_mask16(w[j], 0x0A0A0A0Au) & vmask;
            nl = __builtin_popcount(nlm);
            if (fmt == FMT_FASTA) {
                const uint32_t gtm = eq_mask16(w[j], 0x3E3E3E3Eu) & vmask;
                const uint32_t any = nlm | gtm;
                if (any) mk = (gtm >> (31 - __builtin_clz(any))) & 1 ? 2u : 1u;
            }
        }
        for (int d = 32; d >= 1; d >>= 1) nl += __shfl_xor(nl, d, 64);
        uint32_t tag = mk ? ((uint32_t)tid << 2) | mk : 0;
        for (int d = 32; d >= 1; d >>= 1) tag = max(tag, (uint32_t)__shfl_xor(tag, d, 64));
        if ((tid & 63) == 0) {
            s_nl[j][tid >> 6] = nl;
            s_mk[j][tid >> 6] = tag;
        }
    }
    __syncthreads();
    if (tid < TPB && t0 + tid < ntiles) {
        const int j = tid;
        uint32_t tn = 0, tm = 0;
        for (int q = 0; q < TILE_THREADS / 64; q++) {
            tn += s_nl[j][q];
            tm = max(tm, s_mk[j][q]);
        }
        // (the thread's own copies of tile j's fields: j == tid, registers indexed by the
        // unrolled loop's constant via a select chain)
        ChunkDesc c = cd[0];
        uint64_t r = rel[0];
        uint32_t v = valid[0], a = avail[0];
#pragma unroll
        for (int q = 1; q < TPB; q++)
            if (q == j) {
                c = cd[q];
                r = rel[q];
                v = valid[q];
                a = avail[q];
            }
        TileInfo ti;
        ti.nl = tn;
        ti.valid = v;
        ti.marker = (uint8_t)(tm & 3);
        ti.first = r == 0;
        ti.bh = (uint8_t)c.bh;
        ti.pad = 0;
        ti.avail = a;
        ti.src = c.src_off + r;
        tiles[t0 + j] = ti;
    }
}

// --------------------------------------------------------------------------------
// tile scan, two levels:
//   kept(t)  = valid - (FASTA ? nl : 0) + first   (one break symbol per chunk start)
//              (+ nl << 40 for FASTQ: the line count rides along)
//   hs_in(t) = first ? bh : hs_out(t-1);  hs_out = marker ? (marker == '>') : hs_in
// The header-state recurrence is a "last defining tile" scan (a chunk start or a
// marker defines the state): transform code 0 = identity, 1 = state 0, 2 = state 1.
// --------------------------------------------------------------------------------
constexpr int TSCAN = 1024;
constexpr int FQ_SHIFT = 40;
constexpr uint64_t FQ_MASK = (1ULL << FQ_SHIFT) - 1;
DEV uint64_t tile_kept(const TileInfo& ti, int fmt) {
    const uint64_t kept = ti.valid - (fmt == FMT_FASTA ? ti.nl : 0) + ti.first;
    return fmt == FMT_FASTQ ? kept + ((uint64_t)ti.nl << FQ_SHIFT) : kept;
}
DEV uint32_t tile_tr(const TileInfo& ti) { return ti.marker ? (ti.marker == 2 ? 2u : 1u) : (ti.first ? (ti.bh ? 2u : 1u) : 0u); }

// block-wide inclusive scans over 1024 threads (sum, last non-zero)
DEV void block_scan_1024(unsigned long long& sum, uint32_t& tr) {
    __shared__ unsigned long long s_s[TSCAN / 64];
    __shared__ uint32_t s_t[TSCAN / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long os = __shfl_up(sum, d, 64);
        const uint32_t ot = __shfl_up(tr, d, 64);
        if (lane >= d) {
            sum += os;
            if (!tr) tr = ot;
        }
    }
    if (lane == 63) { s_s[wid] = sum; s_t[wid] = tr; }
    __syncthreads();
    unsigned long long base = 0;
    uint32_t btr = 0;
    for (int w = 0; w < wid; w++) {
        base += s_s[w];
        if (s_t[w]) btr = s_t[w];
    }
    sum += base;
    if (!tr) tr = btr;
}

__global__ __launch_bounds__(TSCAN) void k_tscan_block(const TileInfo* __restrict__ tiles, uint64_t ntiles, int fmt,
                                                      TileOut* __restrict__ touts, TileOut* __restrict__ agg) {
    const uint64_t t = (uint64_t)blockIdx.x * TSCAN + threadIdx.x;
    TileInfo ti{};
    if (t < ntiles) ti = tiles[t];
    const unsigned long long kept = t < ntiles ? tile_kept(ti, fmt) : 0;
    const uint32_t tr0 = t < ntiles ? tile_tr(ti) : 0;
    unsigned long long sum = kept;
    uint32_t tr = tr0;
    block_scan_1024(sum, tr);
    // exclusive values for this tile
    const unsigned long long ex_sum = sum - kept;
    uint32_t ex_tr = __shfl_up(tr, 1, 64);
    __shared__ uint32_t s_last[TSCAN / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 63) s_last[wid] = tr;
    __syncthreads();
    if (lane == 0) ex_tr = wid ? s_last[wid - 1] : 0;
    if (t < ntiles) {
        TileOut to;
        to.out_off = ex_sum;
        to.hs_in = ex_tr;  // transform code, resolved against the block prefix in k_emit
        to.pad = 0;
        touts[t] = to;
    }
    if (threadIdx.x == TSCAN - 1) {
        TileOut a;
        a.out_off = sum;
        a.hs_in = tr;
        a.pad = 0;
        agg[blockIdx.x] = a;
    }
}

// single workgroup: exclusive scan of the block aggregates -> block prefixes
__global__ __launch_bounds__(TSCAN) void k_tscan_top(TileOut* __restrict__ agg, uint64_t nblk, int fmt,
                                                    DevCounters* __restrict__ ctr) {
    __shared__ unsigned long long s_carry;
    __shared__ uint32_t s_tr;
    if (threadIdx.x == 0) { s_carry = 0; s_tr = 0; }
    __syncthreads();
    for (uint64_t base = 0; base < nblk; base += TSCAN) {
        const uint64_t i = base + threadIdx.x;
        TileOut a{};
        if (i < nblk) a = agg[i];
        unsigned long long sum = i < nblk ? a.out_off : 0;
        uint32_t tr = i < nblk ? a.hs_in : 0;
        const unsigned long long mine = sum;
        block_scan_1024(sum, tr);
        const unsigned long long carry = s_carry;
        const uint32_t ctr_in = s_tr;
        // exclusive transform: inclusive of the previous thread
        __shared__ uint32_t s_inc[TSCAN];
        s_inc[threadIdx.x] = tr;
        __syncthreads();
        uint32_t ex_tr = threadIdx.x ? s_inc[threadIdx.x - 1] : 0;
        if (!ex_tr) ex_tr = ctr_in;
        if (i < nblk) {
            TileOut p;
            p.out_off = carry + sum - mine;
            p.hs_in = ex_tr == 2 ? 1u : 0u;  // state entering the block (block 0: tile 0 is a chunk start)
            p.pad = 0;
            agg[i] = p;
        }
        __syncthreads();
        if (threadIdx.x == TSCAN - 1) {
            s_carry = carry + sum;
            if (tr) s_tr = tr;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) ctr->stream_len = fmt == FMT_FASTQ ? (s_carry & FQ_MASK) : s_carry;
}

// --------------------------------------------------------------------------------
// k_zero_edges: k_emit stores a tile's interior words of the packed stream and ORs its two
// edge words (shared with the neighbouring tiles); only those need to start at zero (the
// stream itself is not cleared: ~600 MB per 1.6 GB batch).  One thread per tile.
// --------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_zero_edges(const TileInfo* __restrict__ tiles,
                                                    const TileOut* __restrict__ touts,
                                                    const TileOut* __restrict__ bpre, uint64_t ntiles, int fmt,
                                                    uint64_t* __restrict__ pk, uint32_t* __restrict__ bk) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= ntiles) return;
    const TileInfo ti = tiles[t];
    const uint64_t gsum = bpre[t / TSCAN].out_off + touts[t].out_off;
    const uint64_t g0 = fmt == FMT_FASTQ ? (gsum & FQ_MASK) : gsum;
    const uint64_t total = tile_kept(ti, fmt) & FQ_MASK;  // the symbols k_emit writes
    if (total == 0) return;
    if (g0 & 31) {
        pk[g0 >> 5] = 0;
        bk[g0 >> 5] = 0;
    }
    if ((g0 + total) & 31) {
        pk[(g0 + total - 1) >> 5] = 0;
        bk[(g0 + total - 1) >> 5] = 0;
    }
}

// --------------------------------------------------------------------------------
// k_emit: bytes -> packed 2-bit symbols + break bits, 16 bytes per thread in SWAR:
// byte classes as 16-bit masks, the FASTA header state as a doubling scan over the
// thread's markers, FASTA newlines squeezed out of the 2-bit code word, then the
// thread's (at most 16) symbols land in one or two words of the tile's LDS image.
// --------------------------------------------------------------------------------
DEV uint32_t swap_pairs(uint32_t x) { return ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1); }
// tiles per k_emit workgroup: with every tile's loads issued before the first funnel shift
// (load16_issue / load16_finish), 2 tiles take tokenize 1.31 -> 1.27 ms on C2; 4 tiles, and the
// tiles' phases merged under one set of barriers, gained nothing (1.34 / 1.27 ms;
// profiles/r05_ab_tokenizer_loads.txt)
constexpr int EMIT_TPB = 2;

// one tile's symbols into the tile's LDS image (s_pk / s_bk, zeroed) and out: w = the thread's
// 16 bytes (vh of them valid); s_wsum / s_wmk: per-wave scratch of this tile
DEV void emit_tile(const TileInfo& ti, const TileOut& to, const TileOut& bp, int fmt, const uint32_t (&w)[4],
                   uint32_t vh, unsigned long long* s_pk, uint32_t* s_bk, uint32_t* s_wsum, uint32_t* s_wmk,
                   uint64_t* __restrict__ pk, uint32_t* __restrict__ bk) {
    const uint64_t gsum = bp.out_off + to.out_off;
    const uint64_t g0 = fmt == FMT_FASTQ ? (gsum & FQ_MASK) : gsum;  // global index of the tile's first symbol
    uint32_t hs_in = to.hs_in ? (to.hs_in == 2 ? 1u : 0u) : bp.hs_in;
    if (ti.first) hs_in = ti.bh;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bool fasta = fmt == FMT_FASTA;
    const uint32_t vmask = vh >= 16 ? 0xFFFFu : ((1u << vh) - 1);
    const uint32_t nlm = eq_mask16(w, 0x0A0A0A0Au) & vmask, gtm = eq_mask16(w, 0x3E3E3E3Eu) & vmask;
    // A/C/G/T in either case: the 2-bit code ((b >> 1) ^ (b >> 2)) & 3 names the only
    // letter the byte can be; v_perm looks that letter up and the byte must equal it
    uint32_t acgt = 0, L = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t code = ((w[i] >> 1) ^ (w[i] >> 2)) & 0x03030303u;
        const uint32_t expect = __builtin_amdgcn_perm(0u, 0x74676361u, code);  // "acgt"[code]
        acgt |= flags4(zero_bytes((w[i] | 0x20202020u) ^ expect)) << (4 * i);
        uint32_t x = (code | (code >> 6)) & 0x000F000Fu;
        x = (x | (x >> 12)) & 0xFFu;
        L |= x << (8 * i);  // symbol j at bits 2j, 2j+1
    }
    uint32_t state = 0;
    uint32_t hdr = 0;
    if (fasta) {
        const uint32_t any = nlm | gtm;
        const uint32_t mk = any ? ((gtm >> (31 - __builtin_clz(any))) & 1 ? 2u : 1u) : 0u;
        const uint32_t incl = wave_incl_last(mk);
        if (lane == 63) s_wmk[wid] = incl;
        __syncthreads();
        uint32_t excl = __shfl_up(incl, 1, 64);
        if (lane == 0) excl = 0;
        if (excl == 0)
            for (int ww = wid - 1; ww >= 0; ww--)
                if (s_wmk[ww]) { excl = s_wmk[ww]; break; }
        state = excl ? (excl == 2 ? 1u : 0u) : hs_in;
        // header state per byte: value of the last marker at or before it ('>' 1, '\n' 0)
        uint32_t D = any, V = gtm;
#pragma unroll
        for (int s2 = 1; s2 < 16; s2 <<= 1) {
            V = ((D & V) | (~D & (V << s2))) & 0xFFFFu;
            D = (D | (D << s2)) & 0xFFFFu;
        }
        hdr = (D & V) | (~D & (state ? 0xFFFFu : 0u));
    } else if (fmt == FMT_FASTQ) {
        // line of my first byte: newlines before the tile + before me in the tile, mod 4
        const uint32_t nl = __builtin_popcount(nlm);
        const uint32_t incl = wave_incl_sum(nl);
        if (lane == 63) s_wmk[wid] = incl;
        __syncthreads();
        uint32_t line = (uint32_t)(gsum >> FQ_SHIFT) + incl - nl;
        for (int ww = 0; ww < wid; ww++) line += s_wmk[ww];
        // bytes on a line other than the sequence line (line 1) are breaks
        uint32_t seq = 0, m = nlm, b0 = 0;
        line &= 3;
        while (true) {
            const uint32_t e = m ? (uint32_t)__builtin_ctz(m) : 16u;
            if (line == 1) seq |= ((1u << e) - 1) & ~((1u << b0) - 1);
            if (!m) break;
            b0 = e + 1;
            line = (line + 1) & 3;
            m &= m - 1;
        }
        hdr = ~seq & 0xFFFFu;
    }
    const uint32_t keptm = fasta ? (vmask & ~nlm) : vmask;
    uint32_t brk = (hdr | ~acgt) & 0xFFFFu;
    // squeeze the removed FASTA newlines out of the code and break words
    uint32_t rm = fasta ? nlm : 0u;
    uint64_t L64 = L;
    while (rm) {
        const uint32_t p = 31 - __builtin_clz(rm);
        L64 = (L64 & ((1ull << (2 * p)) - 1)) | ((L64 >> (2 * p + 2)) << (2 * p));
        brk = (brk & ((1u << p) - 1)) | ((brk >> (p + 1)) << p);
        rm ^= 1u << p;
    }
    const uint32_t kept = __builtin_popcount(keptm);
    const uint32_t incl = wave_incl_sum(kept);
    if (lane == 63) s_wsum[wid] = incl;
    __syncthreads();
    uint32_t pos = incl - kept + ti.first;
    uint32_t total = ti.first;
    for (int ww = 0; ww < TILE_THREADS / 64; ww++) {
        if (ww < wid) pos += s_wsum[ww];
        total += s_wsum[ww];
    }
    if (total == 0) return;  // (uniform over the workgroup)
    const uint64_t wbase = g0 >> 5;
    const uint32_t o0 = (uint32_t)(g0 & 31) + pos;  // slot of my first symbol, relative to wbase
    const uint32_t wa = o0 >> 5, r = o0 & 31;
    if (kept) {
        const uint32_t lm = kept >= 16 ? 0xFFFFFFFFu : ((1u << (2 * kept)) - 1);
        const uint32_t Bs = swap_pairs(__builtin_bitreverse32((uint32_t)L64 & lm));  // symbol 0 at bits 31:30
        const uint32_t Bk = __builtin_bitreverse32(brk & ((1u << kept) - 1));       // symbol 0 at bit 31
        uint64_t pa, pb;
        if (r <= 16) {
            pa = (uint64_t)Bs << (32 - 2 * r);
            pb = 0;
        } else {
            pa = (uint64_t)Bs >> (2 * r - 32);
            pb = (uint64_t)Bs << (96 - 2 * r);
        }
        const uint64_t kx = ((uint64_t)Bk << 32) >> r;
        const uint32_t ba = (uint32_t)(kx >> 32), bb = (uint32_t)kx;
        if (pa) atomicOr(&s_pk[wa], (unsigned long long)pa);
        if (ba) atomicOr(&s_bk[wa], ba);
        if (pb) atomicOr(&s_pk[wa + 1], (unsigned long long)pb);
        if (bb) atomicOr(&s_bk[wa + 1], bb);
    }
    if (ti.first && tid == 0) atomicOr(&s_bk[0], 1u << (31 - (uint32_t)(g0 & 31)));  // chunk-start break
    __syncthreads();
    // the tile's words: interior ones are ours alone, the two edge words are shared
    const uint32_t nw = (uint32_t)(((g0 & 31) + total + 31) >> 5);
    for (uint32_t i = tid; i < nw; i += TILE_THREADS) {
        const uint64_t gw = wbase + i;
        const bool edge = (i == 0 && (g0 & 31)) || (i == nw - 1 && ((g0 + total) & 31));
        if (edge) {
            if (s_pk[i]) atomicOr((unsigned long long*)(pk + gw), s_pk[i]);
            if (s_bk[i]) atomicOr(bk + gw, s_bk[i]);
        } else {
            pk[gw] = s_pk[i];
            bk[gw] = s_bk[i];
        }
    }
}

// TPB consecutive tiles per workgroup: every thread's loads for all of them (tile info, scan
// outputs, then its 16 bytes of each tile) are issued before the first tile is emitted
template <int TPB>
__global__ __launch_bounds__(TILE_THREADS) void k_emit(const uint8_t* __restrict__ src,
                                                       const TileInfo* __restrict__ tiles,
                                                       const TileOut* __restrict__ touts,
                                                       const TileOut* __restrict__ bpre, uint64_t ntiles, int fmt,
                                                       uint64_t* __restrict__ pk, uint32_t* __restrict__ bk) {
    constexpr int NW = TILE / 32 + 2;  // output words a tile can touch
    __shared__ unsigned long long s_pk[TPB][NW];
    __shared__ uint32_t s_bk[TPB][NW];
    __shared__ uint32_t s_wsum[TPB][TILE_THREADS / 64];
    __shared__ uint32_t s_wmk[TPB][TILE_THREADS / 64];  // FASTA: last marker per wave; FASTQ: newlines per wave
    const uint64_t t0 = (uint64_t)blockIdx.x * TPB;
    const int tid = threadIdx.x;
    TileInfo ti[TPB];
    TileOut to[TPB], bp[TPB];
#pragma unroll
    for (int j = 0; j < TPB; j++) {
        if (t0 + j < ntiles) {
            ti[j] = tiles[t0 + j];
            to[j] = touts[t0 + j];
            bp[j] = bpre[(t0 + j) / TSCAN];
        } else {
            ti[j] = TileInfo{};
            to[j] = bp[j] = TileOut{};
        }
    }
    const uint32_t my0 = tid * 16;
    uint32_t w[TPB][4], vh[TPB], x[TPB][5];
#pragma unroll
    for (int j = 0; j < TPB; j++) {  // every tile's dword loads first (load16_issue)
        vh[j] = ti[j].valid > my0 ? min(ti[j].valid - my0, 16u) : 0;
        if (vh[j] && load16_fast(ti[j].avail - my0)) load16_issue(src + ti[j].src + my0, x[j]);
    }
#pragma unroll
    for (int j = 0; j < TPB; j++) {
        w[j][0] = w[j][1] = w[j][2] = w[j][3] = 0;
        if (vh[j]) load16_finish(src + ti[j].src + my0, ti[j].avail - my0, x[j], w[j]);
    }
    for (int i = tid; i < TPB * NW; i += TILE_THREADS) {
        (&s_pk[0][0])[i] = 0;
        (&s_bk[0][0])[i] = 0;
    }
#pragma unroll
    for (int j = 0; j < TPB; j++)
        if (t0 + j < ntiles)  // (uniform)
            emit_tile(ti[j], to[j], bp[j], fmt, w[j], vh[j], s_pk[j], s_bk[j], s_wsum[j], s_wmk[j], pk, bk);
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
hipError_t launch_tokenize(const uint8_t* src, uint64_t ntiles, const ChunkDesc* d_chunks, int n_chunks, int fmt,
                           TileInfo* tiles, TileOut* touts, TileOut* tblk, PackedView sv, uint64_t sym_bound,
                           DevCounters* ctr, hipStream_t s) {
    (void)sym_bound;
    const uint64_t nblk = (ntiles + TSCAN - 1) / TSCAN;
    if (n_chunks <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_tile_map, dim3((unsigned)n_chunks), dim3(256), 0, s, d_chunks, tiles);
    hipLaunchKernelGGL(k_tile_summary_m<4>, dim3((unsigned)((ntiles + 3) / 4)), dim3(TILE_THREADS), 0, s, src,
                       d_chunks, ntiles, fmt, tiles);
    hipLaunchKernelGGL(k_tscan_block, dim3((unsigned)nblk), dim3(TSCAN), 0, s, tiles, ntiles, fmt, touts, tblk);
    hipLaunchKernelGGL(k_tscan_top, dim3(1), dim3(TSCAN), 0, s, tblk, nblk, fmt, ctr);
    hipLaunchKernelGGL(k_zero_edges, dim3((unsigned)((ntiles + 255) / 256)), dim3(256), 0, s, tiles, touts, tblk,
                       ntiles, fmt, sv.pk, sv.bk);
    hipLaunchKernelGGL(k_emit<EMIT_TPB>, dim3((unsigned)((ntiles + EMIT_TPB - 1) / EMIT_TPB)), dim3(TILE_THREADS), 0, s,
                       src, tiles, touts, tblk, ntiles, fmt, sv.pk, sv.bk);
    return hipGetLastError();
}

hipError_t launch_synth(uint8_t* dst, uint64_t first_read, uint64_t n_reads, uint64_t seed, uint64_t genome_len,
                        uint32_t read_len, uint32_t wrap, double err_rate, double n_rate, const kc_synth_skew* sk,
                        hipStream_t s) {
    kc_synth_params p{};
    if (sk) {
        p.homo_frac = sk->homo_frac;
        p.dinuc_frac = sk->dinuc_frac;
        p.repeat_len = sk->repeat_len;
        p.repeat_copies = sk->repeat_copies;
    }
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
