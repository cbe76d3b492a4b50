// kc_count_impl.h -- canonical k-mer insertion, Bloom passes and the table dump.
// Included by kc_count_w.hip, which is compiled once per key width W (-DKC_W=1..15).
//
// The reference inserts every window with process_kmer_MT (kmer_hash_table.cpp:
// 2207-2567): a CAS-probed table shared by all threads.  Two MI355X paths produce the
// same table contents:
//
//  direct       k_count<W,MODE>: roll windows, canonicalise, CAS-claim / atomic-add
//               in HBM.  One scattered device-scope atomic per window, so it runs at
//               the chip's scattered-atomic rate (~20 G/s measured); used for small
//               batches (and for the Bloom passes of small batches / the reference
//               filter layout).
//  partitioned  keys are moved to where they are counted instead:
//               p1  windows -> F1 coarse bins (hash prefix), LDS counting sort per tile
//                   so every bin is written as a contiguous run (segmented, one pass);
//               p2f each coarse bin -> its F2 regions, same scheme;
//               p3  one workgroup per region: the region's 64 KiB of buckets in LDS
//                   (zero-filled when the table is fresh), its keys inserted with LDS
//                   atomics, the region written back.
//               Bandwidth-bound (~(4W+1)*8 bytes of key traffic per window plus the
//               table sweeps) instead of atomic-bound.  The Bloom pass runs the same
//               levels on table key word 0 with k_b3 (64 KiB filter regions) as level
//               3; the counting pass behind the filter gates at level 3 (k_p3<..GATE>).
//  merge        shard records (multi-GPU) go through the partitioned levels, or, when
//               they arrive region-sorted, straight to level 3 (k_run_bounds + k_p3).
//
// Table layout (both paths): 128-byte buckets, keys [S][W] u64 then counts [S] u64,
// S = 16/(W+1).  Keys are stored as table keys (kc_common.h: word 0 = a bijective mix,
// never 0, so 0 is EMPTY).  A key lives in the region given by the top bits of word 0;
// its probe sequence starts at the bucket given by the next 9 bits and wraps inside
// the region.  W > 1 keys: word 0 claimed by CAS, other words
// stored, then READY|1 added to the count word; readers matching word 0 wait for READY.
#pragma once
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "kc_common.h"

namespace kc {

static __constant__ uint64_t c_bf_seeds[MAX_NH] = {2411, 3253, 1061, 1129, 2269, 7309, 3491, 8237, 6359, 8779};

// --------------------------------------------------------------------------------
// direct insert of one table key into the HBM table
// --------------------------------------------------------------------------------
template <int W>
DEV bool table_insert(const TableView& tv, const uint64_t (&tk)[W], uint64_t add = 1) {
    constexpr int S = BUCKET_WORDS / (W + 1);
    const uint64_t region = region_of(tk[0], tv.R);
    uint32_t b = bucket_in_region(tk[0], tv.R);
    for (int probe = 0; probe < BPR; probe++) {
        uint64_t* bk = tv.buckets + (region * BPR + b) * BUCKET_WORDS;
        uint64_t w0[S];
        if constexpr (W == 1) {
            const uint4* b4 = reinterpret_cast<const uint4*>(bk);
#pragma unroll
            for (int q = 0; q < S / 2; q++) {
                uint4 v = b4[q];
                w0[2 * q] = ((uint64_t)v.y << 32) | v.x;
                w0[2 * q + 1] = ((uint64_t)v.w << 32) | v.z;
            }
        } else {
#pragma unroll
            for (int s = 0; s < S; s++) w0[s] = bk[s * W];
        }
        int s = 0;
        while (s < S) {
            uint64_t* kp = bk + s * W;
            uint64_t* cp = bk + S * W + s;
            uint64_t v0 = w0[s];
            if (v0 == EMPTY) {
                const uint64_t old = atomicCAS((unsigned long long*)kp, (unsigned long long)EMPTY,
                                               (unsigned long long)tk[0]);
                if (old == EMPTY) {
                    if constexpr (W == 1) {
                        atomicAdd((unsigned long long*)cp, (unsigned long long)add);
                    } else {
#pragma unroll
                        for (int i = 1; i < W; i++) atomic_store_agent(kp + i, tk[i]);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // words land before READY
                        atomicAdd((unsigned long long*)cp, (unsigned long long)(READY + add));
                    }
                    return true;
                }
                v0 = old;
                w0[s] = old;
            }
            if (v0 == tk[0]) {
                if constexpr (W == 1) {
                    atomicAdd((unsigned long long*)cp, (unsigned long long)add);
                    return true;
                } else {
                    const uint64_t c = atomic_load_agent(cp);
                    if (!(c & READY)) continue;  // claimed, not yet published: retry this slot
                    asm volatile("" ::: "memory");
                    bool eq = true;
#pragma unroll
                    for (int i = 1; i < W; i++) eq &= atomic_load_agent(kp + i) == tk[i];
                    if (eq) {
                        atomicAdd((unsigned long long*)cp, (unsigned long long)add);
                        return true;
                    }
                }
            }
            s++;
        }
        b = (b + 1) & (BPR - 1);
    }
    return false;  // region full
}

// --------------------------------------------------------------------------------
// Bloom filter: both filters interleaved in one bit array (filter-1 bit of h = 2h,
// filter-2 bit = 2h+1, the MyAtomicBitArrayFT layout, mybitarray.hpp:30-125)
// --------------------------------------------------------------------------------
struct BloomLocal {
    uint32_t new_first, new_second, failed;
};

// Two layouts of the k-mer's positions:
//  reference (KC_BLOOM_LAYOUT=reference; mybitarray + calculate_hashes,
//    double_bloomfilter.hpp:276-281): h_j = XXH64(root, seed_j) & (bits - 1), root = the
//    strand-symmetric Rabin-Karp hash mod 2^54: n independent random words, filter-1 bit
//    of h at 2h and filter-2 bit at 2h+1 (MyAtomicBitArrayFT, mybitarray.hpp:30-125).
//  blocked (the default): a split-block filter.  Each k-mer owns one 64-byte block of 16
//    words: words 0-7 hold filter 1, words 8-15 filter 2 (the same 2 x 256 bits per block
//    as the interleaved bit array).  Position j sets bit b_j = bits 5j..5j+4 of
//    bmix(t0) in word j mod 8 of each filter, so the positions of one k-mer lie in
//    distinct words (no repeats for ceil(hf) <= 8) and a test is two 16-byte reads and
//    a shift per position.  The block is picked by the top bits of the k-mer's table key
//    word 0 t0 (kc_common.h to_tkey, a bijective mix of the canonical key): block =
//    ((t0 >> 32) * blocks) >> 32, the same hash prefix as the table's region index, so a
//    filter region of BF_BLOCKS_PER_REGION blocks is one contiguous 64 KiB slice that the
//    partitioned Bloom pass holds in LDS (k_b3), and the filter-2 words of a table
//    region's keys are one contiguous slice its level 3 copies to LDS for the gate
//    (k_p3<..., GATE>).  The filter only gates, so either layout gives the reference's
//    counts for every k-mer seen at least twice.
constexpr int BF_BLOCK_WORDS = 16;               // 512 bits: filter 1 in words 0-7, filter 2 in 8-15
// ((t0 >> 32) * nblocks) >> 32 for the power-of-two block count: a shift (the count is
// uniform, so its log2 is scalar work)
DEV uint64_t bloom_block(uint64_t t0, uint64_t nblocks) { return (t0 >> 32) >> (32 - __builtin_ctzll(nblocks)); }
// position hash: t0 is already a strong mix of the key (to_tkey), one multiply-fold
// spreads its low bits (which vary inside a block) over all position fields
DEV uint64_t bmix(uint64_t t0) {
    const uint64_t x = (t0 ^ 0xD6E8FEB86659FD93ULL) * 0xBF58476D1CE4E5B9ULL;
    return x ^ (x >> 31);
}
// bit of position j (word j & 7 of a filter): 5-bit fields, six per 32-bit half of h (no
// field straddles the halves, so each is one bit-field extract)
DEV uint32_t sb_bit(uint64_t h, int j) {
    return j < 6 ? ((uint32_t)h >> (5 * j)) & 31 : ((uint32_t)(h >> 32) >> (5 * (j - 6))) & 31;
}
// the 8 words of one filter of a block (16-byte aligned) into registers
DEV void load8(const uint32_t* p, uint32_t (&w)[8]) {
    const uint4 a = reinterpret_cast<const uint4*>(p)[0], b = reinterpret_cast<const uint4*>(p)[1];
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}
// all of the first n positions set in the 8 words f (one filter of a block): the bits of
// all MAX_NH positions gathered branch-free (two extracts and a shift-or each), then masked
DEV bool sb_all(const uint32_t (&f)[8], uint64_t h, int n) {
    uint32_t got = 0;
#pragma unroll
    for (int j = 0; j < MAX_NH; j++) got |= ((f[j & 7] >> sb_bit(h, j)) & 1) << j;
    const uint32_t need = (1u << n) - 1;
    return (got & need) == need;
}

// insertion_process (double_bloomfilter.hpp:371-413) on one block of the blocked layout;
// `blk` is the block in HBM (direct pass) or in LDS (k_b3).  A "set" counts as ours only
// if our atomicOr flipped the bit (MyAtomicBitArrayFT::set, mybitarray.hpp:87-125).
// Positions j >= 8 share word j - 8 and count once if they repeat its bit.
// unique: the key is inserted by no other thread at the same time (pre-aggregated records,
// kc_bloom_records_device), so a filter-1 bit it needed that another thread set meanwhile was
// set by ANOTHER key: as if that key had come first.  The insertion then counts as the
// key's first sighting unless every missing bit was set by others (the filter was complete
// for it, as a sequential pass would have found it); the reference's rule -- any such bit
// sends the key to filter 2 -- is for concurrent sightings of one key (windows), and applied
// to a batch of distinct keys it sent a third of the singletons to filter 2
DEV void block_insert(uint32_t* blk, uint64_t t0, int nh, BloomLocal& loc, bool unique = false) {
    const uint64_t h = bmix(t0);
    uint32_t f1[8], f2[8];
    load8(blk + 8, f2);
    load8(blk, f1);  // (with filter 2: one wait for the block's 64 bytes instead of two in turn)
    if (sb_all(f2, h, nh)) return;  // in the second filter already
    // the key's positions as one bit mask per filter word (a position j >= 8 that repeats the bit
    // of position j - 8 merges with it: counted once); n = distinct positions, s1 / s2 = those set
    uint32_t pm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < MAX_NH; j++)
        if (j < nh) pm[j & 7] |= 1u << sb_bit(h, j);
    int n = 0, s1 = 0, s2 = 0;
#pragma unroll
    for (int w = 0; w < 8; w++) {
        n += __popc(pm[w]);
        s1 += __popc(pm[w] & f1[w]);
        s2 += __popc(pm[w] & f2[w]);
    }
    // a filter's missing bits set by four 64-bit atomic ORs (word pairs; a pair with nothing to
    // set ORs zero), issued back to back: one wait for all of them.  (One 32-bit atomic per
    // position under its own branch waited for each return in turn.)  mine = bits this thread
    // flipped, as MyAtomicBitArrayFT::set counts them
    auto set_missing = [&](uint32_t* f, const uint32_t (&fw)[8]) {
        uint64_t m[4], old[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            m[q] = (uint64_t)(pm[2 * q] & ~fw[2 * q]) | (uint64_t)(pm[2 * q + 1] & ~fw[2 * q + 1]) << 32;
            old[q] = atomicOr(reinterpret_cast<unsigned long long*>(f) + q, (unsigned long long)m[q]);
        }
        int mine = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) mine += __popcll(m[q] & ~old[q]);
        return mine;
    };
    bool to_second = true;
    if (s1 != n) {
        const int mine = set_missing(blk, f1);
        if (mine == n - s1 || (unique && mine > 0)) { loc.new_first++; to_second = false; }
        else loc.failed++;
    }
    if (to_second) {
        const int mine = set_missing(blk + 8, f2);
        if (unique || mine == n - s2) loc.new_second++;  // (a distinct key was not in filter 2 before)
    }
}

// pass-2 gate: all of the first trunc(hf) filter-2 bits set (parallel_parser.hpp:
// 2436-2441); f2 = the block's 8 filter-2 words (HBM, or the LDS slice of k_p3)
DEV bool block_gate(const uint32_t* f2, uint64_t t0, int nh_gate) {
    uint32_t w[8];
    load8(f2, w);
    return sb_all(w, bmix(t0), nh_gate);
}
// blocks [lo, hi] hold the filter of table region r's keys (region_of and bloom_block
// are monotone in the same 32-bit hash prefix)
DEV void region_blocks(uint64_t r, uint64_t R, uint64_t nblocks, uint64_t& lo, uint64_t& hi) {
    const uint64_t h_lo = ((r << 32) + R - 1) / R;                               // first prefix of r
    const uint64_t h_hi = min((((r + 1) << 32) + R - 1) / R, 1ULL << 32) - 1;   // last prefix of r
    lo = (h_lo * nblocks) >> 32;
    hi = (h_hi * nblocks) >> 32;
}

// reference layout: word and bit (of the filter-1 bit; filter 2 is the next bit) of the
// first n hash functions of a root
template <int N>
DEV void ref_slots(const BloomView& bf, uint64_t root, int n, uint64_t (&widx)[N], uint32_t (&bpos)[N]) {
#pragma unroll
    for (int j = 0; j < N; j++)
        if (j < n) {
            const uint64_t bit = 2 * (xxh64_u64(root, c_bf_seeds[j]) & bf.mask);
            widx[j] = bit >> 5;
            bpos[j] = (uint32_t)(bit & 31);
        }
}

DEV uint32_t* bloom_block_ptr(const BloomView& bf, uint64_t t0) {
    return bf.bits + bloom_block(t0, bf.nblocks) * BF_BLOCK_WORDS;
}

// insertion_process on the HBM filter (direct pass 1): root for the reference layout, the
// table key word t0 for the blocked one
DEV void bloom_insert(const BloomView& bf, uint64_t root, uint64_t t0, BloomLocal& loc) {
    if (bf.blocked) {
        block_insert(bloom_block_ptr(bf, t0), t0, bf.nh, loc);
        return;
    }
    uint64_t widx[MAX_NH];
    uint32_t bpos[MAX_NH];
    uint32_t view[MAX_NH];
    int s1 = 0, s2 = 0;
    ref_slots(bf, root, bf.nh, widx, bpos);
#pragma unroll
    for (int j = 0; j < MAX_NH; j++)
        if (j < bf.nh) view[j] = bf.bits[widx[j]];
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

DEV bool bloom_gate(const BloomView& bf, uint64_t root, uint64_t t0) {
    if (bf.blocked) return block_gate(bloom_block_ptr(bf, t0) + 8, t0, bf.nh_gate);
    uint64_t widx[MAX_NH];
    uint32_t bpos[MAX_NH];
    ref_slots(bf, root, bf.nh_gate, widx, bpos);
    bool all = true;
#pragma unroll
    for (int j = 0; j < MAX_NH; j++)
        if (j < bf.nh_gate) all &= (bf.bits[widx[j]] >> (bpos[j] + 1)) & 1;
    return all;
}

// block reduction of up to 4 counters, one atomic each per block
DEV void block_add4(unsigned long long v0, unsigned long long v1, unsigned long long v2, unsigned long long v3,
                    unsigned long long* d0, unsigned long long* d1, unsigned long long* d2,
                    unsigned long long* d3) {
    __shared__ unsigned long long s_red[4][16];  // up to 1024-thread blocks
    unsigned long long v[4] = {v0, v1, v2, v3};
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
        for (int w = 0; w < (int)(blockDim.x / 64); w++) x += s_red[threadIdx.x][w];
        unsigned long long* dst = threadIdx.x == 0 ? d0 : threadIdx.x == 1 ? d1 : threadIdx.x == 2 ? d2 : d3;
        if (x && dst) atomicAdd(dst, x);
    }
}

// --------------------------------------------------------------------------------
// windows of a tile
// --------------------------------------------------------------------------------
// per-thread windows of one tile (the tile is COUNT_THREADS * run_w windows):
// kc_internal.h run_width (shared with the host's partition sizing)
template <int W>
constexpr int run_w() { return run_width(W); }
template <int W>
constexpr int tile_win() { return COUNT_THREADS * run_w<W>(); }
// the segmented (single-pass) level 1: kc_internal.h scatter_threads
template <int W>
constexpr int scatter_threads() { return scatter_threads_w(W); }
// windows per thread of k_p1<W, ..., NT> (the segmented launch: p1_runw; the 256-thread exact
// levels: run_w) and its LDS before the heavy table: the bins' arrays and the tile of OW-word keys
template <int W, int NT>
constexpr int k1_runw() { return NT == scatter_threads_w(W) ? p1_runw(W) : run_w<W>(); }
template <int W, int OW, int NT>
constexpr size_t p1_smem(uint32_t F) { return bin_lds_bytes(F) + (size_t)NT * k1_runw<W, NT>() * 8 * OW; }
// the segmented k_p1's LDS stage of the packed stream: two buffers of the words a tile reads
// (kc_internal.h p1_stage_words), 8 + 4 bytes per word, after the heavy table
template <int W, int NT>
constexpr int k1_stage_words() { return NT * k1_runw<W, NT>() / 32 + W + 3; }
template <int W, int NT>
constexpr size_t p1_stage_smem() { return (size_t)k1_stage_words<W, NT>() * 24; }
// Level 2 runs one 1024-thread workgroup per CU for keys of up to two words: twice the
// tile of level 1 (16384 one-word keys, 128 KiB of LDS) halves the barriers per key and
// doubles the runs each bin gets per tile (C2: k_p2f 5.6 -> 5.0 ms on one box); wider
// keys take smaller groups so that the tile still fits the LDS
template <int W>
constexpr int p2f_threads() { return p2f_threads_w(W); }

// table key of the window ending at p (MODE 0 path: direct extraction)
template <int W>
DEV bool window_tkey(const PackedView& sv, uint64_t p, const RollConst& rk, uint64_t (&tk)[W]) {
    uint64_t fwd[W], rc[W], key[W];
    if (!extract_window<W>(sv, p, rk, fwd)) return false;
    revcomp<W>(fwd, rk, rc);
    canonical<W>(fwd, rc, key);
    to_tkey<W>(key, tk);
    return true;
}

// MODE 1/2: the Bloom root (RollingHasherDual mod 2^54) is a rolled quantity, so these
// modes roll one contiguous run of run_w windows per thread.
template <int W, int RUNW = run_w<W>(), class F>
DEV void tile_rolled(const PackedView& sv, uint64_t t0, uint64_t t1, const RollConst& rk, F&& f) {
    const uint64_t r0 = t0 + (uint64_t)threadIdx.x * RUNW, r1 = min(r0 + RUNW, t1);
    if (r0 < r1) {
        const uint64_t ps = r0 >= (uint64_t)(rk.k - 1) ? r0 - (rk.k - 1) : 0;
        roll_run<W, true>(sv, ps, r0, r1, rk, f);
    }
}

// --------------------------------------------------------------------------------
// k_count<W, MODE>: direct path. MODE 0 count, 1 Bloom pass 1, 2 count behind the gate
// --------------------------------------------------------------------------------
template <int W, int MODE>
__global__ __launch_bounds__(COUNT_THREADS) void k_count(PackedView sv, int k, TableView tv, BloomView bf,
                                                         DevCounters* __restrict__ ctr, uint64_t pow5_k,
                                                         uint64_t pow5_km1) {
    constexpr int TW = tile_win<W>();
    const uint64_t M = ctr->stream_len;
    const uint64_t t0 = (uint64_t)blockIdx.x * TW;
    uint32_t n_win = 0, n_ins = 0, n_fail = 0;
    BloomLocal bl = {0, 0, 0};
    if (t0 < M) {
        const uint64_t t1 = min(t0 + TW, M);
        const RollConst rk = make_roll<W>(k, pow5_k, pow5_km1);
        if constexpr (MODE == 0) {
            constexpr int RUNW = run_w<W>();
            const uint64_t r0 = t0 + (uint64_t)threadIdx.x * RUNW;
            if (r0 < t1)
                run_windows<W, RUNW>(sv, r0, t1, rk,
                                     [&](int, bool valid, const uint64_t (&fwd)[W], const uint64_t (&rc)[W]) {
                    if (!valid) return;
                    uint64_t key[W], tk[W];
                    canonical<W>(fwd, rc, key);
                    to_tkey<W>(key, tk);
                    n_win++;
                    n_ins++;
                    if (!table_insert<W>(tv, tk)) n_fail++;
                });
        } else {
            tile_rolled<W>(sv, t0, t1, rk, [&](const uint64_t (&fwd)[W], const uint64_t (&rc)[W], uint64_t root) {
                n_win++;
                uint64_t key[W], tk[W];
                canonical<W>(fwd, rc, key);
                to_tkey<W>(key, tk);
                if constexpr (MODE == 1) {
                    bloom_insert(bf, root, tk[0], bl);
                } else {
                    if (!bloom_gate(bf, root, tk[0])) return;
                    n_ins++;
                    if (!table_insert<W>(tv, tk)) n_fail++;
                }
            });
        }
    }
    if constexpr (MODE == 1)
        block_add4(n_win, bl.new_first, bl.new_second, bl.failed, &ctr->bf_windows, &ctr->new_in_first,
                   &ctr->new_in_second, &ctr->failed_in_first);
    else
        block_add4(n_win, n_ins, n_fail, 0, &ctr->windows, &ctr->inserted, &ctr->overflow, nullptr);
}

// --------------------------------------------------------------------------------
// partitioned path
// --------------------------------------------------------------------------------
// LDS of a scatter pass: hist, start, lim, sp (u32 x F), gbase (u64 x F), then the keys
constexpr size_t hist_smem(uint32_t F) { return bin_lds_bytes(F); }
template <int W, int NT = COUNT_THREADS>
constexpr size_t part_smem(uint32_t F) {
    return hist_smem(F) + (size_t)NT * run_w<W>() * 8 * W;
}

// exclusive scan of an LDS u32 array of n entries by one NT-thread block
template <int NT = COUNT_THREADS>
DEV void block_excl_scan_lds(const uint32_t* in, uint32_t* out, uint32_t n) {
    __shared__ uint32_t s_w[NT / 64];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t per = (n + NT - 1) / NT;
    const uint32_t lo = min(n, tid * per), hi = min(n, lo + per);
    uint32_t sum = 0;
    for (uint32_t i = lo; i < hi; i++) sum += in[i];
    const uint32_t incl = wave_incl_sum(sum);
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    uint32_t base = incl - sum;
    for (int w = 0; w < wid; w++) base += s_w[w];
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t v = in[i];
        out[i] = base;
        base += v;
    }
    __syncthreads();
}

// LDS of a scatter: per bin its tile count, its first tile slot, the tile slots that
// fit its output (lim), the destination of its next key (gbase; during a tile's write-out
// it holds destination minus tile slot, and the tile's end turns it back into the next
// destination: 24 bytes per bin, which is what lets big tables keep wide bins at both
// levels); then the tile's keys
struct PartLds {
    uint32_t* hist;
    uint32_t* start;
    uint32_t* lim;
    uint32_t* sp;  // keys past the output's end: count, then offset in the tile's spill allocation
    uint64_t* gbase;
    uint64_t* keys;
};
DEV PartLds part_lds(uint8_t* smem, uint32_t F) {
    PartLds l;
    l.hist = reinterpret_cast<uint32_t*>(smem);
    l.start = l.hist + F;
    l.lim = l.start + F;
    l.sp = l.lim + F;
    l.gbase = reinterpret_cast<uint64_t*>(l.sp + F);
    l.keys = l.gbase + F + (F & 1);  // 16-byte aligned
    return l;
}

// bin of a table key: its region bin (table levels) or its shard owner (routing);
// the kind is a template parameter so the table levels carry no routing branch.
struct BinRegion {  // level-1 bin (coarse: region >> f2bits) or level-2 bin (region & mask)
    static constexpr bool kOwner = false;
    uint64_t R;
    int f2bits;
    uint32_t mask;
    int coarse;
    DEV uint32_t operator()(uint64_t t0) const {
        const uint32_t r = __umulhi((uint32_t)(t0 >> 32), (uint32_t)R);  // region_of
        return coarse ? r >> f2bits : r & mask;
    }
};
// level 1 always takes coarse bins: a copy with the mode known at compile time spares the
// select between both bin formulas in every bin computation of k_p1 (three per key)
DEV BinRegion level1_bins(const BinRegion& b) { return BinRegion{b.R, b.f2bits, b.mask, 1}; }
struct BinOwner {
    static constexpr bool kOwner = true;
    uint32_t parts;
    DEV uint32_t operator()(uint64_t t0) const { return owner_of(t0, parts); }
};
DEV BinOwner level1_bins(const BinOwner& b) { return b; }

// Where a scatter pass writes bin b.  Exact layout: one contiguous run per bin at offsets
// from a histogram pass + scan.  Segmented layout (single pass, no histogram): a
// fixed-capacity segment per (bin, producing workgroup); keys that would pass a
// segment's end are dropped and raise DevCounters::part_overflow, and the exact
// pipeline then redoes the batch (launched behind a device-side gate).
struct OutExact {
    static constexpr bool kSeg = false;
    DEV uint64_t room(uint32_t, uint64_t) const { return ~0ULL; }  // keys bin b can still take
};
struct OutSeg {
    static constexpr bool kSeg = true;
    uint64_t stride;  // keys between the segments of bins b and b+1
    uint64_t base;    // first key of bin 0's segment for this workgroup
    uint64_t cap;     // keys per segment
    // keys past a segment's end: appended to the batch's skew list (inserted after level 3 by
    // the exact pipeline); count passes append {key words, 1} records (the list also takes the
    // heavy records of repeated windows), the Bloom pass plain keys.  A full list raises the
    // batch's overflow flag (whole-batch redo).
    uint64_t* spill;
    uint64_t spill_cap;
    unsigned long long* spill_n;
    unsigned long long* overflow;
    int rec;
    DEV uint64_t start(uint32_t b) const { return (uint64_t)b * stride + base; }
    DEV uint64_t room(uint32_t b, uint64_t gbase) const {
        const uint64_t end = start(b) + cap;
        return gbase < end ? end - gbase : 0;
    }
};

// key-stream loads and stores (nontemporal forms measured no faster: r01_v11_ab_nontemporal.txt)
DEV uint64_t ks_load(const uint64_t* p) { return *p; }
DEV void ks_store(uint64_t* p, uint64_t v) { *p = v; }

// rank of this lane among the set lanes of a wave mask
DEV uint32_t lane_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// wave-aggregated append: the lanes with `want` get consecutive slots of a list (one atomic
// per wave); returns the slot (or ~0 for lanes without `want`)
DEV uint64_t wave_append(bool want, unsigned long long* counter) {
    const uint64_t m = __ballot(want);
    if (!m) return ~0ULL;
    const int leader = __builtin_ctzll(m);
    unsigned long long base = 0;
    if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(counter, (unsigned long long)__popcll(m));
    base = __shfl(base, leader, 64);
    return want ? base + lane_rank(m) : ~0ULL;
}
// Counting-sort the tile's keys (in registers: tk[j] valid where ok[j]) by bin into
// LDS and write each bin as one contiguous run at gbase[bin].  The rank of a key inside
// its bin comes back from the histogram atomic, so one LDS atomic per key suffices.
// Returns true if a segmented run did not fit.
struct NoMid {
    DEV void operator()() const {}
};
// mid(): called once the tile's keys are in LDS (tk / ok are dead from there on: a caller
// may load its next tile into them)
template <int W, int RUNW, class Bin, class Out, int NT = COUNT_THREADS, class Mid = NoMid>
DEV bool scatter_tile(const PartLds& l, uint32_t F, const Bin& bin, const Out& o, uint64_t (&tk)[RUNW][W],
                      bool (&ok)[RUNW], uint64_t* __restrict__ out, Mid&& mid = Mid()) {
    __shared__ unsigned long long s_spbase;
    __shared__ uint32_t s_spills;  // some bin of the tile spills (set by the setup, read after a barrier)
    const int tid = threadIdx.x;
    uint32_t rank[RUNW];  // (the bins are recomputed below: one multiply, fewer registers)
    if (Out::kSeg && tid == 0) s_spills = 0;
#pragma unroll
    for (int j = 0; j < RUNW; j++) rank[j] = ok[j] ? atomicAdd(&l.hist[bin(tk[j][0])], 1u) : 0;
    __syncthreads();
    block_excl_scan_lds<NT>(l.hist, l.start, F);
#pragma unroll
    for (int j = 0; j < RUNW; j++)
        if (ok[j]) {
            const uint32_t slot = l.start[bin(tk[j][0])] + rank[j];
#pragma unroll
            for (int w = 0; w < W; w++) l.keys[slot * W + w] = tk[j][w];
        }
    // per bin: destination minus tile slot, the tile slots that fit the bin's output, and
    // the keys past its end
    bool spills = false;
    for (uint32_t b = tid; b < F; b += NT) {
        const uint32_t st = l.start[b], h = l.hist[b];
        const uint64_t g = l.gbase[b];
        const uint32_t fit = (uint32_t)min((uint64_t)h, o.room(b, g));
        l.gbase[b] = g - st;  // destination minus tile slot (modulo 2^64) until the tile's end
        l.lim[b] = st + fit;
        l.sp[b] = h - fit;
        spills |= fit < h;
    }
    if (Out::kSeg && spills) s_spills = 1;
    mid();
    __syncthreads();
    if constexpr (Out::kSeg) {
        if (s_spills) {
            // one allocation in the skew list for all the tile's spilled keys (a bin's spilled
            // keys are the tail of its run in the tile)
            const uint32_t last = l.sp[F - 1];
            block_excl_scan_lds<NT>(l.sp, l.sp, F);
            if (tid == 0) s_spbase = atomicAdd(o.spill_n, (unsigned long long)(l.sp[F - 1] + last));
            __syncthreads();
        }
    }
    const uint32_t n = l.start[F - 1] + l.hist[F - 1];
    for (uint32_t i = tid; i < n; i += NT) {
        uint64_t key[W];
#pragma unroll
        for (int w = 0; w < W; w++) key[w] = l.keys[i * W + w];
        const uint32_t b = bin(key[0]);
        const uint32_t lim = l.lim[b];
        if (i < lim) {
            const uint64_t dst = l.gbase[b] + i;
#pragma unroll
            for (int w = 0; w < W; w++) ks_store(out + dst * W + w, key[w]);
        } else if constexpr (Out::kSeg) {
            const uint64_t pos = s_spbase + l.sp[b] + (i - lim);
            if (pos < o.spill_cap) {
                uint64_t* r = o.spill + pos * (W + o.rec);
#pragma unroll
                for (int w = 0; w < W; w++) r[w] = key[w];
                if (o.rec) r[W] = 1;
            } else {
                atomicOr(o.overflow, 1ULL);
            }
        }
    }
    __syncthreads();
    for (uint32_t b = tid; b < F; b += NT) {
        l.gbase[b] += l.lim[b];  // past the keys written (a segment's fill never passes its end)
        l.hist[b] = 0;
    }
    __syncthreads();
    return false;
}

// The segmented scatter of k_p1 and k_p2f, as a pipelined tile loop: three barriers per tile
// instead of scatter_tile's six.  The write-out of tile t and the window arithmetic + rank
// atomics of tile t+1 are not separated by a barrier (they touch disjoint LDS: keys / lim /
// gbase / sp against registers / hist), so one wave's VALU work overlaps another's stores.
// Per tile:
//   rank atomics (hist was cleared by the previous tile's setup)              barrier 1
//   wave 0: exclusive scan of hist -> start and the tile's key count           barrier 2
//   placement into keys[]; per-bin setup (advances the previous tile's fill,
//     clears hist); mid() (the caller may load its next tile into tk / ok)     barrier 3
//   (a bin past its segment's end: one skew-list allocation for the tile)
//   write-out
// Before the first tile: hist = 0, lim = 0, gbase = each bin's first destination
// (scatter_seg_init); after the last: a barrier, then a bin's next destination is
// gbase + lim (scatter_seg_next).
DEV void scatter_seg_init(const PartLds& l, uint32_t b, uint64_t first) {
    l.hist[b] = 0;
    l.lim[b] = 0;
    l.gbase[b] = first;
}
DEV uint64_t scatter_seg_next(const PartLds& l, uint32_t b) { return l.gbase[b] + l.lim[b]; }

// Where a scatter's write-out puts a key: W words at out[dst] (StoreWords), or a level-2
// record of 6 bytes (StoreRec6: one-word keys in tables of >= 2^16 regions, k_p2f -> k_p3).
struct StoreWords {
    template <int W>
    DEV void operator()(uint64_t* __restrict__ out, uint64_t dst, const uint64_t (&key)[W], uint32_t) const {
#pragma unroll
        for (int w = 0; w < W; w++) ks_store(out + dst * W + w, key[w]);
    }
};
// Level-2 record of a one-word key (table key word 0 = x << 32 | lo): the region r holding it
// fixes x to [xlo(r), xlo(r + 1)), xlo(r) = ceil(r 2^32 / R), a range of at most 2^16 values
// when R >= 2^16, so a record is lo (32 bits) and d = x - xlo(r) (16 bits): 6 instead of 8
// bytes per key for k_p2f to write and k_p3 to read.  Records go in pairs of three dwords
// {lo_even, lo_odd, d_even | d_odd << 16} (one stream per segment; record p of the key array
// at byte 6p, since segment starts are multiples of 8 records).
DEV uint64_t region_xlo(uint64_t r, uint64_t R) { return ((r << 32) + R - 1) / R; }
struct StoreRec6 {
    const uint32_t* xlo;  // LDS: xlo of each bin's region
    DEV void operator()(uint64_t* __restrict__ out, uint64_t dst, const uint64_t (&key)[1], uint32_t b) const {
        uint32_t* q = reinterpret_cast<uint32_t*>(out) + (dst >> 1) * 3;
        q[dst & 1] = (uint32_t)key[0];
        reinterpret_cast<uint16_t*>(q + 2)[dst & 1] = (uint16_t)((uint32_t)(key[0] >> 32) - xlo[b]);
    }
};
// pre(): called after the rank atomics (k_p1 issues the loads of its next tile's words there)
// Level record of a two-word key (kc_internal.h PartBufs.rec12): table key (t0, t1) with
// t0 = x << 32 | lo, t1 = key word 0 (2k - 64 bits) | TK_FLAG.  Three dwords {lo, t1 low, t1 bits
// 32.. (hb = 2k - 96, or 0) | flag << hb | (x mod 2^xb) << (hb + 1)}: 12 instead of 16 bytes when
// hb + 1 + xb <= 32.  The record's bin spans fewer than 2^xb values of x from its lowest, x0, so
// x = x0 + ((x - x0) mod 2^xb) is recovered from x mod 2^xb: x0 = bin << xb in a power-of-two
// geometry (the Bloom pass's fine bins), region_xlo of the bin's first region in the table's
// (R12_REG).  The host checks the spans (k <= 51 at level 1 of >= 2^7 bins; k <= 55 at level 2
// of >= 2^16 regions).
struct Rec12 {
    int hb, xb;
    DEV uint3 enc(uint64_t t0, uint64_t t1) const {
        const uint32_t x = (uint32_t)(t0 >> 32), d = x & ((1u << xb) - 1);
        const uint32_t hi = ((uint32_t)(t1 >> 32) & ((1u << hb) - 1)) | (uint32_t)((t1 >> 62) & 1) << hb;
        return make_uint3((uint32_t)t0, (uint32_t)t1, hi | d << (hb + 1));
    }
    DEV void dec(uint3 r, uint32_t x0, uint64_t& t0, uint64_t& t1) const {
        const uint32_t x = x0 + (((r.z >> (hb + 1)) - x0) & ((1u << xb) - 1));
        t0 = ((uint64_t)x << 32) | r.x;
        t1 = ((uint64_t)(r.z & ((1u << hb) - 1)) << 32) | r.y | ((uint64_t)((r.z >> hb) & 1) << 62);
    }
};
// two-word keys as 12-byte records (rec12) or whole keys: the format a uniform branch inside one
// scatter loop (a loop instantiated per format kept both copies' invariants live, and the level
// 2 of two-word keys spilled them, each reload waiting for the tile's prefetch loads)
struct StoreW2 {
    bool rec12;
    Rec12 rc;
    DEV void operator()(uint64_t* __restrict__ out, uint64_t dst, const uint64_t (&key)[2], uint32_t) const {
        if (rec12) {
            reinterpret_cast<uint3*>(out)[dst] = rc.enc(key[0], key[1]);
        } else {
            ks_store(out + dst * 2, key[0]);
            ks_store(out + dst * 2 + 1, key[1]);
        }
    }
};

template <int W, int RUNW, class Bin, class Out, int NT, class Mid = NoMid, class St = StoreWords, class Pre = NoMid>
DEV void scatter_seg(const PartLds& l, uint32_t F, const Bin& bin, const Out& o, uint64_t (&tk)[RUNW][W],
                     bool (&ok)[RUNW], uint64_t* __restrict__ out, Mid&& mid = Mid(),
                     const St& store = St(), Pre&& pre = Pre()) {
    static_assert(NT * RUNW <= 65536, "ranks ride in 16 bits");
    __shared__ unsigned long long s_spbase;
    __shared__ uint32_t s_spills, s_n;
    const int tid = threadIdx.x, lane = tid & 63;
    uint32_t pk[RUNW];  // bin << 16 | rank in the bin, ~0 = no key
#pragma unroll
    for (int j = 0; j < RUNW; j++) {
        const uint32_t b = bin(tk[j][0]);
        if constexpr (W >= 2) {
            // every slot issues its rank atomic (adding 0 where there is no key; a bin is in range
            // for any key word), so the RUNW atomics go out back to back with one wait for their
            // returns; an atomic under `if (ok)` was waited for inside the branch.  (One-word keys
            // keep the branch: their level 1 has no registers left for RUNW returns in flight.)
            const uint32_t rk = atomicAdd(&l.hist[b], ok[j] ? 1u : 0u);
            pk[j] = ok[j] ? (b << 16) | rk : ~0u;
        } else {
            pk[j] = ok[j] ? (b << 16) | atomicAdd(&l.hist[b], 1u) : ~0u;
        }
    }
    pre();
    __syncthreads();  // 1
    if (tid < 64) {
        if (F % 4 == 0) {  // (hist and start 16-byte aligned) four bins per 16-byte LDS access
            const uint32_t per = (F / 4 + 63) / 64, lo = min(F / 4, lane * per), hi = min(F / 4, lo + per);
            const uint4* h4 = reinterpret_cast<const uint4*>(l.hist);
            uint4* s4 = reinterpret_cast<uint4*>(l.start);
            uint32_t sum = 0;
#pragma unroll 1
            for (uint32_t i = lo; i < hi; i++) {
                const uint4 v = h4[i];
                sum += v.x + v.y + v.z + v.w;
            }
            const uint32_t incl = wave_incl_sum(sum);
            uint32_t run = incl - sum;
#pragma unroll 1
            for (uint32_t i = lo; i < hi; i++) {
                const uint4 v = h4[i];
                s4[i] = make_uint4(run, run + v.x, run + v.x + v.y, run + v.x + v.y + v.z);
                run += v.x + v.y + v.z + v.w;
            }
            if (lane == 63) s_n = incl;
        } else {
            const uint32_t per = (F + 63) / 64, lo = min(F, lane * per), hi = min(F, lo + per);
            uint32_t sum = 0;
#pragma unroll 1
            for (uint32_t i = lo; i < hi; i++) sum += l.hist[i];
            const uint32_t incl = wave_incl_sum(sum);
            uint32_t run = incl - sum;
#pragma unroll 1
            for (uint32_t i = lo; i < hi; i++) {
                l.start[i] = run;
                run += l.hist[i];
            }
            if (lane == 63) s_n = incl;
        }
        if (Out::kSeg && lane == 0) s_spills = 0;
    }
    __syncthreads();  // 2
#pragma unroll
    for (int j = 0; j < RUNW; j++)
        if (pk[j] != ~0u) {
            const uint32_t slot = l.start[pk[j] >> 16] + (pk[j] & 0xFFFFu);
#pragma unroll
            for (int w = 0; w < W; w++) l.keys[slot * W + w] = tk[j][w];
        }
    bool spills = false;
#pragma unroll 1
    for (uint32_t b = tid; b < F; b += NT) {
        const uint32_t st = l.start[b], h = l.hist[b];
        const uint64_t g = l.gbase[b] + l.lim[b];  // the bin's next destination
        const uint32_t fit = (uint32_t)min((uint64_t)h, o.room(b, g));
        l.gbase[b] = g - st;  // destination minus tile slot (modulo 2^64) during the write-out
        l.lim[b] = st + fit;
        l.sp[b] = h - fit;
        l.hist[b] = 0;
        spills |= fit < h;
    }
    if (Out::kSeg && spills) s_spills = 1;
    mid();
    __syncthreads();  // 3
    if constexpr (Out::kSeg) {
        if (s_spills) {
            // one allocation in the skew list for all the tile's spilled keys (a bin's spilled
            // keys are the tail of its run in the tile)
            const uint32_t last = l.sp[F - 1];
            block_excl_scan_lds<NT>(l.sp, l.sp, F);
            if (tid == 0) s_spbase = atomicAdd(o.spill_n, (unsigned long long)(l.sp[F - 1] + last));
            __syncthreads();
        }
    }
    const uint32_t n = s_n;
    auto emit = [&](uint32_t i, const uint64_t (&key)[W], uint32_t b, uint32_t lim, uint64_t g) {
        if (i < lim) {
            store(out, g + i, key, b);
        } else if constexpr (Out::kSeg) {
            const uint64_t pos = s_spbase + l.sp[b] + (i - lim);
            if (pos < o.spill_cap) {
                uint64_t* r = o.spill + pos * (W + o.rec);
#pragma unroll
                for (int w = 0; w < W; w++) r[w] = key[w];
                if (o.rec) r[W] = 1;
            } else {
                atomicOr(o.overflow, 1ULL);
            }
        }
    };
    // two keys per thread per round, their LDS reads issued together
#pragma unroll 1
    for (uint32_t i0 = tid; i0 < n; i0 += 2 * NT) {
        const uint32_t i1 = i0 + NT;
        const bool has1 = i1 < n;
        uint64_t k0[W], k1[W];
#pragma unroll
        for (int w = 0; w < W; w++) {
            k0[w] = l.keys[i0 * W + w];
            k1[w] = l.keys[(has1 ? i1 : i0) * W + w];
        }
        const uint32_t b0 = bin(k0[0]), b1 = bin(k1[0]);
        const uint32_t lim0 = l.lim[b0], lim1 = l.lim[b1];
        const uint64_t g0 = l.gbase[b0], g1 = l.gbase[b1];
        emit(i0, k0, b0, lim0, g0);
        if (has1) emit(i1, k1, b1, lim1, g1);
    }
}

// MODE 3 and 5 are Bloom pass 1 (MODE 5 writes the whole table key: its level-1 output is
// kept for the counting pass, kc_api.cpp "level-1 reuse")
constexpr bool bloom_mode(int MODE) { return MODE == 3 || MODE == 5; }

// Repeated windows (homopolymer runs: poly-A tails, poly-G artefacts; dinucleotide
// microsatellites).  One key repeated millions of times would send all its copies into one
// level-2 segment and one level-3 region (SURVEY 7 "hard parts"; the reference's hot spot is
// the increase_count CAS, kmer.cpp:699).  A window equal to a neighbour one or two windows
// away (within the thread's run) leaves the key stream and is counted in a small LDS table
// of the workgroup (the heavy table: HT keys with their counts); at the end of the
// workgroup's range every entry becomes one {key, count} record of the batch's skew list,
// inserted after level 3.  The Bloom pass keeps two copies of such a key instead
// (insertion_process changes nothing after a k-mer's second insertion,
// double_bloomfilter.hpp:371-413).  Waves without a repeat skip it after one ballot.
constexpr int HT = 64;  // heavy-table entries per workgroup
template <int OW>
constexpr size_t heavy_smem() { return (size_t)HT * (OW + 1) * 8; }
struct HeavyTab {
    uint64_t* keys;  // HT x OW words (word 0 == 0: empty)
    uint64_t* cnt;   // HT counts (READY | count once the key words are published)
};
template <int OW>
DEV HeavyTab heavy_tab(uint8_t* p) {
    HeavyTab h;
    h.keys = reinterpret_cast<uint64_t*>(p);
    h.cnt = h.keys + HT * OW;
    return h;
}
DEV void heavy_clear(const HeavyTab& h, int words) {
    for (int i = threadIdx.x; i < HT * words; i += blockDim.x) h.keys[i] = 0;
}
// add `add` windows of key into the table (all lanes of the wave call it; `active` lanes
// insert).  Lanes whose key finds no room return true: the caller appends them to the list.
template <int OW>
DEV bool heavy_insert(const HeavyTab& h, const uint64_t (&key)[OW], bool active, uint64_t add) {
    uint32_t e = (uint32_t)((key[0] * 0x9E3779B97F4A7C15ULL) >> 58) & (HT - 1);
    int probes = 0;
    bool done = !active, full = false;
    while (__ballot(!done)) {
        if (!done) {
            uint64_t* kp = h.keys + e * OW;
            uint64_t w0 = __hip_atomic_load(kp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            bool next = false;
            if (w0 == EMPTY) {
                const uint64_t old = atomicCAS(reinterpret_cast<unsigned long long*>(kp), 0ULL,
                                               (unsigned long long)key[0]);
                if (old == EMPTY) {  // claimed: publish the other words, then the count
#pragma unroll
                    for (int w = 1; w < OW; w++)
                        __hip_atomic_store(kp + w, key[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    atomicAdd(reinterpret_cast<unsigned long long*>(h.cnt + e), (unsigned long long)(READY + add));
                    done = true;
                }  // lost the slot: read it again
            } else if (w0 == key[0]) {
                const uint64_t c = __hip_atomic_load(h.cnt + e, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (c & READY) {
                    bool eq = true;
#pragma unroll
                    for (int w = 1; w < OW; w++) eq &= kp[w] == key[w];
                    if (eq) {
                        atomicAdd(reinterpret_cast<unsigned long long*>(h.cnt + e), (unsigned long long)add);
                        done = true;
                    } else {
                        next = true;
                    }
                }  // not published yet: read it again
            } else {
                next = true;
            }
            if (next) {
                e = (e + 1) & (HT - 1);
                if (++probes >= HT) {
                    full = true;
                    done = true;
                }
            }
        }
    }
    return full;
}
// append {key, count} records (count passes) or count (<= 2) plain keys (Bloom pass) to the
// batch's skew list, one list allocation per wave
template <int OW, int MODE>
DEV void skew_append(const PartBufs& pb, DevCounters* ctr, bool want, const uint64_t (&key)[OW], uint64_t c) {
    const uint32_t copies = !want ? 0u : bloom_mode(MODE) ? (c >= 2 ? 2u : 1u) : 1u;
    uint32_t incl = wave_incl_sum(copies);
    const uint32_t total = __shfl(incl, 63, 64);
    if (!total) return;
    unsigned long long base = 0;
    if ((threadIdx.x & 63) == 0) base = atomicAdd(&ctr->spill_n, (unsigned long long)total);
    base = __shfl(base, 0, 64);
    for (uint32_t q = 0; q < copies; q++) {
        const uint64_t pos = base + incl - copies + q;
        if (pos >= pb.spill_cap) {
            atomicOr(&ctr->part_overflow, 1ULL);
            break;
        }
        uint64_t* r = pb.spill + pos * (bloom_mode(MODE) ? OW : OW + 1);
#pragma unroll
        for (int w = 0; w < OW; w++) r[w] = key[w];
        if (!bloom_mode(MODE)) r[OW] = c;
    }
}

template <int OW, int RUNW, int MODE>
DEV void combine_repeats(uint64_t (&tk)[RUNW][OW], bool (&ok)[RUNW], const HeavyTab& h, const PartBufs& pb,
                         DevCounters* ctr) {
    // repeated windows (lane masks only in the common case): equal to the next window
    // (homopolymer) or to the one after ((CA)n)
    uint32_t rep = 0;
#pragma unroll
    for (int j = 0; j + 1 < RUNW; j++) {
        bool e1 = ok[j] && ok[j + 1], e2 = j + 2 < RUNW && ok[j] && ok[j + 2];
#pragma unroll
        for (int w = 0; w < OW; w++) {
            e1 = e1 && tk[j][w] == tk[j + 1][w];
            if (j + 2 < RUNW) e2 = e2 && tk[j][w] == tk[j + 2][w];
        }
        if (e1) rep |= 3u << j;
        if (e2) rep |= 5u << j;
    }
    if (__ballot(rep != 0) == 0) return;
    // window slot by window slot, the lanes holding a repeat there insert it (no LDS staging:
    // the tile's key area may still be read by another wave's write-out, scatter_seg)
#pragma unroll 1
    for (int j = 0; j < RUNW; j++) {  // (not unrolled: one copy of the insertion code)
        const bool act = (rep >> j) & 1;
        if (__ballot(act) == 0) continue;
        uint64_t key[OW];
#pragma unroll
        for (int w = 0; w < OW; w++) key[w] = 0;
#pragma unroll
        for (int q = 0; q < RUNW; q++)
            if (q == j)
#pragma unroll
                for (int w = 0; w < OW; w++) key[w] = tk[q][w];
        const bool full = heavy_insert<OW>(h, key, act, 1);
        skew_append<OW, MODE>(pb, ctr, full, key, 1);
    }
#pragma unroll
    for (int j = 0; j < RUNW; j++)
        if ((rep >> j) & 1) ok[j] = false;
}
// end of a workgroup's range: the heavy table's entries -> records of the skew list
template <int OW, int MODE>
DEV void heavy_flush(const HeavyTab& h, const PartBufs& pb, DevCounters* ctr) {
    __syncthreads();
    if (threadIdx.x < HT) {  // one wave
        const int e = threadIdx.x;
        uint64_t key[OW];
#pragma unroll
        for (int w = 0; w < OW; w++) key[w] = h.keys[e * OW + w];
        const uint64_t c = h.cnt[e] & CNT_MASK;
        const bool has = key[0] != EMPTY;
        skew_append<OW, MODE>(pb, ctr, has, key, c);
        const uint64_t nrec = __ballot(has);
        if (threadIdx.x == 0 && nrec) atomicAdd(&ctr->heavy_n, (unsigned long long)__popcll(nrec));
    }
}

// gated kernels (the exact fallback of a segmented batch) run only if *gate != 0
DEV bool gated_off(const unsigned long long* gate) { return gate && *gate == 0; }

// words per level-1 output key: the Bloom pass (MODE 3) moves table key word 0 only
constexpr int p1_out_words(int W, int MODE) { return MODE == 3 ? 1 : W; }
// The waves per SIMD a scatter kernel can have resident: its LDS tile (NT threads x RUNW keys of
// OW words) bounds the workgroups per CU.  Its launch bound asks for no more (capped by `cap`),
// so the register budget is what that occupancy leaves: wide keys at one workgroup per CU got 64
// VGPRs and 316 bytes of scratch per lane from a bound of 8 waves (C5's level 2) -- registers
// the LDS would never let other waves use
constexpr int scatter_waves(int NT, int RUNW, int OW, int cap) {
    const int wg = (int)(LDS_BYTES / ((size_t)NT * RUNW * 8 * OW));
    const int w = (wg < 1 ? 1 : wg) * NT / 256;
    return w < 1 ? 1 : w > cap ? cap : w;
}


// Level 1: windows of a contiguous symbol range -> coarse bins (region >> f2bits).
// MODE 0: count; 2: count behind the Bloom gate on the rolled root (reference layout);
// 3: Bloom pass 1, blocked layout (keys = t0, bins = filter regions); 4: count, gated
// at level 3 (blocked layout).
// SCATTER = false: histogram only ([bin][block] into hist1); true: write the keys,
// exact layout (offsets off1) or segmented (Out = OutSeg: single pass, the segment
// fill counts go to hist1).  `count`: add windows / inserted to the counters (off for
// the histogram pass of a fallback, whose windows the segmented pass counted already).
template <int W, int MODE, bool SCATTER, class Bin, class Out, int NT = COUNT_THREADS>
__global__ __launch_bounds__(NT, scatter_waves(NT, k1_runw<W, NT>(), p1_out_words(W, MODE), 4)) void k_p1(PackedView sv, int k, BloomView bf,
                                                      DevCounters* __restrict__ ctr, PartBufs pb, uint32_t F, Bin bin_arg,
                                                      uint64_t* __restrict__ out, uint64_t pow5_k, uint64_t pow5_km1,
                                                      Out o, const unsigned long long* gate, int count) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const Bin bin = level1_bins(bin_arg);
    constexpr int RUNW = k1_runw<W, NT>(), TW = NT * RUNW;
    constexpr bool COUNTS = !SCATTER || Out::kSeg;
    constexpr bool ROLLED = MODE == 2;       // gate on the rolled root (reference layout)
    constexpr int OW = p1_out_words(W, MODE);  // words per output key
    if (gated_off(gate)) return;
    if (gate && !SCATTER && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&ctr->part_fallbacks, 1ULL);
    const PartLds l = part_lds(smem, F);
    constexpr bool HEAVY = Out::kSeg && !Bin::kOwner && !ROLLED;  // repeated windows -> heavy table
    const HeavyTab ht = heavy_tab<OW>(smem + p1_smem<W, OW, NT>(F));
    if constexpr (HEAVY) {
        heavy_clear(ht, OW);
        for (int i = threadIdx.x; i < HT; i += NT) ht.cnt[i] = 0;
    }
    const int tid = threadIdx.x;
    const uint64_t M = ctr->stream_len;
    const uint64_t per = ((M + pb.nblk1 - 1) / pb.nblk1 + TW - 1) / TW * TW;
    const uint64_t lo = min(M, (uint64_t)blockIdx.x * per), hi = min(M, lo + per);
    // Segmented count / Bloom passes read a tile's words from an LDS stage: the words of the
    // next tile are loaded while this one is scattered (its rank atomics issue the loads, its
    // placement stores them), so the windows of a tile start without waiting for HBM.  Tile
    // t0 reads words (t0 >> 5) - W - 1 .. (t0 + TW) >> 5 (run_windows, t0 a multiple of 32).
    constexpr bool STAGE = Out::kSeg && !ROLLED;  // the segmented level 1 reads its windows from the LDS stage
    constexpr int SW = k1_stage_words<W, NT>();
    static_assert(!STAGE || SW <= NT, "one stage word per thread");
    uint64_t* st_pk = reinterpret_cast<uint64_t*>(smem + p1_smem<W, OW, NT>(F) + heavy_smem<OW>());
    uint32_t* st_bk = reinterpret_cast<uint32_t*>(st_pk + 2 * SW);
    const uint64_t wlim = M ? ((M - 1) >> 5) + 1 : 0;  // the last word run_windows may read
    auto stage_word = [&](uint64_t ts, int i, uint64_t& pw, uint32_t& bw) {
        const int64_t w = (int64_t)(ts >> 5) - (W + 1) + i;
        const bool in = w >= 0 && (uint64_t)w <= wlim;
        pw = in ? sv.pk[w] : 0;
        bw = in ? sv.bk[w] : 0;
    };
    if constexpr (STAGE)
        if (lo < hi && tid < SW) stage_word(lo, tid, st_pk[tid], st_bk[tid]);
    int par = 0;  // the stage buffer of the current tile
    Out ob = o;
    if constexpr (Out::kSeg) ob.base = (uint64_t)blockIdx.x * o.cap;  // segment (b, block) = b * nblk1 + block
    for (uint32_t b = tid; b < F; b += NT) {
        if constexpr (Out::kSeg) {
            scatter_seg_init(l, b, ob.start(b));
        } else {
            l.hist[b] = 0;
            if constexpr (SCATTER) l.gbase[b] = pb.off1[(uint64_t)b * pb.nblk1 + blockIdx.x];
        }
    }
    __syncthreads();
    const RollConst rk = make_roll<W>(k, pow5_k, pow5_km1);
    uint32_t n_win = 0, n_ins = 0;
    for (uint64_t t0 = lo; t0 < hi; t0 += TW) {
        const uint64_t t1 = min(t0 + TW, hi);
        uint64_t tk[RUNW][OW];
        bool ok[RUNW];
        if constexpr (!ROLLED) {
            const uint64_t r0 = t0 + (uint64_t)tid * RUNW;
#pragma unroll
            for (int j = 0; j < RUNW; j++) ok[j] = false;
            auto emit = [&](int j, bool valid, const uint64_t (&fwd)[W], const uint64_t (&rc)[W]) {
                uint64_t key[W], t[W];
                canonical<W>(fwd, rc, key);
                to_tkey<W>(key, t);
#pragma unroll
                for (int w = 0; w < OW; w++) tk[j][w] = t[w];
                ok[j] = valid;
            };
            if (r0 < t1) {
                if constexpr (STAGE)
                    run_windows_src<W, RUNW>(PkStage{st_pk + par * SW, st_bk + par * SW, (int64_t)(t0 >> 5) - (W + 1)},
                                             r0, t1, rk, emit);
                else
                    run_windows<W, RUNW>(sv, r0, t1, rk, emit);
            }
            if constexpr (COUNTS) {
#pragma unroll
                for (int j = 0; j < RUNW; j++) {
                    n_win += ok[j];
                    n_ins += MODE == 0 ? ok[j] : 0;  // MODE 4: level 3 counts the gated insertions
                }
            }
            if constexpr (HEAVY) combine_repeats<OW, RUNW, MODE>(tk, ok, ht, pb, ctr);
        } else {
            // rolled run: slot j <- the j-th symbol of the thread's run (static indices)
#pragma unroll
            for (int j = 0; j < RUNW; j++) ok[j] = false;
            tile_rolled<W, RUNW>(sv, t0, t1, rk, [&](const uint64_t (&fwd)[W], const uint64_t (&rc)[W], uint64_t root) {
                if constexpr (COUNTS) n_win++;
                uint64_t key[W], t[W];
                canonical<W>(fwd, rc, key);
                to_tkey<W>(key, t);
                if (!bloom_gate(bf, root, t[0])) return;
                if constexpr (COUNTS) n_ins++;
                // at most run_w windows per run: append into the first free register slot
#pragma unroll
                for (int j = 0; j < RUNW; j++)
                    if (!ok[j]) {
                        ok[j] = true;
#pragma unroll
                        for (int w = 0; w < W; w++) tk[j][w] = t[w];
                        break;
                    }
            });
        }
        if constexpr (SCATTER) {
            if constexpr (Out::kSeg) {
                const bool nxt = STAGE && t0 + TW < hi && tid < SW;
                uint64_t npk = 0;
                uint32_t nbk = 0;
                auto mid = [&]() {  // placement phase: the next tile's words into the other buffer
                    if (nxt) {
                        st_pk[(par ^ 1) * SW + tid] = npk;
                        st_bk[(par ^ 1) * SW + tid] = nbk;
                    }
                };
                auto pre = [&]() {  // after the rank atomics: load them
                    if (nxt) stage_word(t0 + TW, tid, npk, nbk);
                };
                if constexpr (OW == 2)  // level 1 as 12-byte records (the kept Bloom levels, the table's)
                    scatter_seg<OW, RUNW, Bin, Out, NT>(l, F, bin, ob, tk, ok, out, mid,
                                                        StoreW2{(pb.rec12 & R12_P1) != 0, Rec12{pb.r12_hb, pb.r12_xb1}},
                                                        pre);
                else
                    scatter_seg<OW, RUNW, Bin, Out, NT>(l, F, bin, ob, tk, ok, out, mid, StoreWords(), pre);
                par ^= 1;
            } else {
                scatter_tile<OW, RUNW, Bin, Out, NT>(l, F, bin, ob, tk, ok, out, NoMid());
            }
        } else {
#pragma unroll
            for (int j = 0; j < RUNW; j++)
                if (ok[j]) atomicAdd(&l.hist[bin(tk[j][0])], 1u);
        }
    }
    if constexpr (!SCATTER) {
        __syncthreads();
        for (uint32_t b = tid; b < F; b += NT) pb.hist1[(uint64_t)b * pb.nblk1 + blockIdx.x] = l.hist[b];
    }
    if constexpr (Out::kSeg) {  // segment fills, once the last write-out has read lim / gbase
        __syncthreads();
        for (uint32_t b = tid; b < F; b += NT)
            pb.hist1[(uint64_t)b * pb.nblk1 + blockIdx.x] = (uint32_t)(scatter_seg_next(l, b) - ob.start(b));
    }
    if constexpr (HEAVY) heavy_flush<OW, MODE>(ht, pb, ctr);
    // routing (owner bins) counts windows here and insertions at the owner; the Bloom
    // pass counts its windows apart
    if constexpr (COUNTS)
        if (count) {
            if constexpr (bloom_mode(MODE))
                block_add4(n_win, 0, 0, 0, &ctr->bf_windows, nullptr, nullptr, nullptr);
            else
                block_add4(n_win, Bin::kOwner ? 0 : n_ins, 0, 0, &ctr->windows, &ctr->inserted, nullptr, nullptr);
        }
}

// Level 1 over a key array (keys received from other shards): [0, n) split over nblk1
// blocks, bins = the coarse bins of the table key.
// Item count on the device (the spill list of a segmented batch): dn != nullptr ->
// n = min(*dn, cap), or 0 once the batch's overflow flag is up (the whole batch is redone).
struct DevN {
    const unsigned long long* dn;
    uint64_t cap;
    const unsigned long long* ovf;
};
DEV uint64_t item_count(uint64_t n, const DevN& d) {
    if (!d.dn) return n;
    return *d.ovf ? 0 : min((uint64_t)*d.dn, d.cap);
}

template <int W, bool SCATTER>
__global__ __launch_bounds__(COUNT_THREADS, 4) void k_p1k(const uint64_t* __restrict__ in, uint64_t n_host, PartBufs pb,
                                                       uint32_t F, BinRegion bin, DevCounters* __restrict__ ctr,
                                                       int cnt_word, DevN dn, int istride) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int RUNW = run_w<W>(), TW = tile_win<W>();
    const uint64_t n = item_count(n_host, dn);
    const PartLds l = part_lds(smem, F);
    const int tid = threadIdx.x;
    const uint64_t per = ((n + pb.nblk1 - 1) / pb.nblk1 + TW - 1) / TW * TW;
    const uint64_t lo = min(n, (uint64_t)blockIdx.x * per), hi = min(n, lo + per);
    for (uint32_t b = tid; b < F; b += COUNT_THREADS) {
        l.hist[b] = 0;
        if constexpr (SCATTER) l.gbase[b] = pb.off1[(uint64_t)b * pb.nblk1 + blockIdx.x];
    }
    __syncthreads();
    uint32_t n_inv = 0;
    unsigned long long added = 0;  // records (cnt_word >= 0): sum of their counts
    for (uint64_t t0 = lo; t0 < hi; t0 += TW) {
        uint64_t tk[RUNW][W];
        bool ok[RUNW];
        uint32_t inr = 0;  // the tile's loads first (past hi: item lo), then their use
#pragma unroll
        for (int q = 0; q < RUNW; q++) {
            const uint64_t i = t0 + tid + (uint64_t)q * COUNT_THREADS;
            const uint64_t ii = i < hi ? i : lo;
            inr |= (uint32_t)(i < hi) << q;
#pragma unroll
            for (int w = 0; w < W; w++) tk[q][w] = in[ii * istride + w];
        }
#pragma unroll
        for (int q = 0; q < RUNW; q++) {
            const bool inq = (inr >> q) & 1;
            ok[q] = inq && tk[q][0] != EMPTY;  // 0 is never a table key: skip (counted as invalid)
            if constexpr (!SCATTER) {
                n_inv += inq & !ok[q];
#pragma unroll
                for (int w = 0; w < W; w++)
                    if (w == cnt_word && ok[q]) added += tk[q][w] & CNT_MASK;
            }
        }
        if constexpr (SCATTER) {
            scatter_tile<W, RUNW>(l, F, bin, OutExact{}, tk, ok, pb.keys1);
        } else {
#pragma unroll
            for (int q = 0; q < RUNW; q++)
                if (ok[q]) atomicAdd(&l.hist[bin(tk[q][0])], 1u);
        }
    }
    if constexpr (!SCATTER) {
        __syncthreads();
        for (uint32_t b = tid; b < F; b += COUNT_THREADS) pb.hist1[(uint64_t)b * pb.nblk1 + blockIdx.x] = l.hist[b];
        if (cnt_word < 0) added = cnt_word == -1 && blockIdx.x == 0 && tid == 0 ? n : 0;  // (-2: counted later)
        if (dn.dn) added = 0;  // spilled windows: counted by level 1 (or at level 3 behind the gate)
        block_add4(added, n_inv, 0, 0, &ctr->inserted, &ctr->invalid, nullptr, nullptr);
    }
}

// direct insert of a key array (small batches)
template <int W>
__global__ __launch_bounds__(COUNT_THREADS) void k_insert_keys(const uint64_t* __restrict__ in, uint64_t n,
                                                               TableView tv, DevCounters* __restrict__ ctr) {
    uint32_t n_fail = 0, n_inv = 0;
    const uint64_t i = (uint64_t)blockIdx.x * COUNT_THREADS + threadIdx.x;
    if (i < n) {
        uint64_t tk[W];
#pragma unroll
        for (int w = 0; w < W; w++) tk[w] = in[i * W + w];
        if (tk[0] == EMPTY) n_inv++;  // 0 is never a table key: skip (counted as invalid)
        else if (!table_insert<W>(tv, tk)) n_fail++;
    }
    block_add4(blockIdx.x == 0 && threadIdx.x == 0 ? n : 0, n_fail, n_inv, 0, &ctr->inserted, &ctr->overflow,
               &ctr->invalid, nullptr);
}

// --------------------------------------------------------------------------------
// shard merge (pre-aggregated sharding): a rank's table -> {table key, count} records
// grouped by owner shard; the owner adds the counts into its own table.
// --------------------------------------------------------------------------------
// one 128-byte bucket into registers: eight 16-byte loads issued together
DEV void load_bucket(const uint64_t* __restrict__ b, uint64_t (&bw)[BUCKET_WORDS]) {
    const uint4* b4 = reinterpret_cast<const uint4*>(b);
    uint4 v[BUCKET_WORDS / 2];
#pragma unroll
    for (int c = 0; c < BUCKET_WORDS / 2; c++) v[c] = b4[c];
#pragma unroll
    for (int c = 0; c < BUCKET_WORDS / 2; c++) {
        bw[2 * c] = ((uint64_t)v[c].y << 32) | v[c].x;
        bw[2 * c + 1] = ((uint64_t)v[c].w << 32) | v[c].z;
    }
}

// SCATTER = false: per-block record counts per owner ([owner][block] into hist);
// true: records {W table-key words, raw count} at off[owner][block] + rank.
template <int W, bool SCATTER>
__global__ __launch_bounds__(256) void k_route_table(TableView tv, uint32_t parts, uint32_t* __restrict__ hist,
                                                     const uint64_t* __restrict__ off, uint64_t* __restrict__ out) {
    constexpr int S = BUCKET_WORDS / (W + 1);
    __shared__ uint32_t s_cnt[RT_MAX_PARTS];
    __shared__ uint64_t s_base[RT_MAX_PARTS];
    const uint32_t nblk = gridDim.x;
    for (uint32_t d = threadIdx.x; d < parts; d += 256) {
        s_cnt[d] = 0;
        if constexpr (SCATTER) s_base[d] = off[(uint64_t)d * nblk + blockIdx.x];
    }
    __syncthreads();
    const uint64_t bkt = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (bkt < tv.nbuckets) {
        uint64_t bw[BUCKET_WORDS];
        load_bucket(tv.buckets + bkt * BUCKET_WORDS, bw);
#pragma unroll
        for (int sl = 0; sl < S; sl++) {
            const uint64_t t0 = bw[sl * W];
            if (t0 == EMPTY) continue;
            const uint32_t d = owner_of(t0, parts);
            const uint32_t r = atomicAdd(&s_cnt[d], 1u);
            if constexpr (SCATTER) {
                uint64_t* o = out + (s_base[d] + r) * (W + 1);
#pragma unroll
                for (int w = 0; w < W; w++) o[w] = bw[sl * W + w];
                o[W] = bw[S * W + sl] & CNT_MASK;
            }
        }
    }
    if constexpr (!SCATTER) {
        __syncthreads();
        for (uint32_t d = threadIdx.x; d < parts; d += 256) hist[(uint64_t)d * nblk + blockIdx.x] = s_cnt[d];
    }
}

// add the counts of {W table-key words, count} records into the table (direct inserts:
// one record per distinct key of a sending shard, far fewer than windows)
template <int W>
__global__ __launch_bounds__(COUNT_THREADS) void k_insert_counts(const uint64_t* __restrict__ rec, uint64_t n,
                                                                 TableView tv, DevCounters* __restrict__ ctr) {
    uint32_t n_fail = 0, n_inv = 0;
    unsigned long long added = 0;
    const uint64_t i = (uint64_t)blockIdx.x * COUNT_THREADS + threadIdx.x;
    if (i < n) {
        uint64_t tk[W];
#pragma unroll
        for (int w = 0; w < W; w++) tk[w] = rec[i * (W + 1) + w];
        const uint64_t c = rec[i * (W + 1) + W] & CNT_MASK;
        if (tk[0] == EMPTY) n_inv++;
        else if (c && !table_insert<W>(tv, tk, c)) n_fail++;
        else added = c;
    }
    block_add4(added, n_fail, n_inv, 0, &ctr->inserted, &ctr->overflow, &ctr->invalid, nullptr);
}

// Level 2: coarse bin c (block = c * B2 + j) -> its F2 regions (next bits of tkey[0]).
template <int W, bool SCATTER>
__global__ __launch_bounds__(COUNT_THREADS, 4) void k_p2(TableView tv, PartBufs pb, const unsigned long long* gate) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int RUNW = run_w<W>(), TW = tile_win<W>();
    if (gated_off(gate)) return;
    const uint32_t F = tv.F2;
    const BinRegion bin{tv.R, tv.f2bits, F - 1, 0};
    const PartLds l = part_lds(smem, F);
    const int tid = threadIdx.x;
    const uint32_t c = blockIdx.x / pb.B2, j = blockIdx.x % pb.B2;
    const uint64_t cs = pb.off1[(uint64_t)c * pb.nblk1], ce = pb.off1[(uint64_t)(c + 1) * pb.nblk1];
    const uint64_t part = (ce - cs + pb.B2 - 1) / pb.B2;
    const uint64_t lo = min(ce, cs + j * part), hi = min(ce, lo + part);
    const uint64_t rbase = (uint64_t)c * F;
    for (uint32_t b = tid; b < F; b += COUNT_THREADS) {
        l.hist[b] = 0;
        if constexpr (SCATTER) l.gbase[b] = pb.off2[(rbase + b) * pb.B2 + j];
    }
    __syncthreads();
    for (uint64_t t0 = lo; t0 < hi; t0 += TW) {
        uint64_t tk[RUNW][W];
        bool ok[RUNW];
#pragma unroll
        for (int q = 0; q < RUNW; q++) {
            const uint64_t i = t0 + tid + (uint64_t)q * COUNT_THREADS;
            ok[q] = i < hi;
            const uint64_t ii = ok[q] ? i : lo;  // (the select on the address: nothing waits for the loads)
#pragma unroll
            for (int w = 0; w < W; w++) tk[q][w] = pb.keys1[ii * W + w];
        }
        if constexpr (SCATTER) {
            scatter_tile<W, RUNW>(l, F, bin, OutExact{}, tk, ok, pb.keys2);
        } else {
#pragma unroll
            for (int q = 0; q < RUNW; q++)
                if (ok[q]) atomicAdd(&l.hist[bin(tk[q][0])], 1u);
        }
    }
    if constexpr (!SCATTER) {
        __syncthreads();
        for (uint32_t b = tid; b < F; b += COUNT_THREADS) pb.hist2[(rbase + b) * pb.B2 + j] = l.hist[b];
    }
}

// Level 2, segmented: coarse bin c's level-1 segments of workgroups [s_lo, s_hi)
// (block = c * B2 + j) -> segments (c * F2 + region, j) of capacity cap2, one pass.
// The input segments are read as one virtual run (exclusive prefix of their fills in
// LDS; each thread walks a monotone segment cursor).
// LDS: the scatter's arrays plus the segment-fill prefix (a level-2 workgroup reads
// ceil(nblk1 / B2) level-1 segments)
template <int W, int NT>
constexpr size_t p2f_smem(uint32_t F, uint32_t nseg_max) { return part_smem<W, NT>(F) + (size_t)(nseg_max + 1) * 4; }

// IS: u64 words per level-1 item (W, or the whole table key of a kept level-1 output when
// the Bloom pass reads only its word 0)
// REC6: write 6-byte level-2 records (StoreRec6) instead of whole keys (one-word keys)
template <int W, int NT, int IS = W, bool REC6 = false>
__global__ __launch_bounds__(NT, scatter_waves(NT, run_w<W>(), W, 2048 / NT > 8 ? 8 : 2048 / NT)) void k_p2f(TableView tv, PartBufs pb, DevCounters* __restrict__ ctr,
                                                          int REC) {
    static_assert(!REC6 || W == 1, "6-byte records hold one-word keys");
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int RUNW = run_w<W>(), TW = NT * RUNW;
    if (ctr->part_overflow) return;  // level 1 overflowed: the exact pipeline redoes the batch
    const uint32_t F = tv.F2;
    const BinRegion bin{tv.R, tv.f2bits, F - 1, 0};
    const PartLds l = part_lds(smem, F);
    uint32_t* pre = reinterpret_cast<uint32_t*>(smem + part_smem<W, NT>(F));
    const int tid = threadIdx.x;
    const uint32_t c = blockIdx.x / pb.B2, j = blockIdx.x % pb.B2;
    const uint32_t s_lo = (uint32_t)((uint64_t)j * pb.nblk1 / pb.B2);
    const uint32_t nseg = (uint32_t)((uint64_t)(j + 1) * pb.nblk1 / pb.B2) - s_lo;
    const uint64_t seg0 = (uint64_t)c * pb.nblk1 + s_lo;  // level-1 segment index of cursor 0
    // output segment of region r: r * B2T + jo (a deferred level 3 keeps several batches' segments)
    const uint32_t B2T = pb.b2t ? pb.b2t : pb.B2, jo = pb.b2off + j;
    const OutSeg o{(uint64_t)B2T * pb.cap2, ((uint64_t)c * F * B2T + jo) * pb.cap2, pb.cap2,
                   pb.spill, pb.spill_cap, &ctr->spill_n, &ctr->part_overflow, REC};
    for (uint32_t i = tid; i <= nseg; i += NT) pre[i] = i < nseg ? pb.hist1[seg0 + i] : 0;
    uint32_t* xlo = pre + nseg + 1;  // REC6: xlo of the F regions of coarse bin c
    if constexpr (REC6)
        for (uint32_t b = tid; b < F; b += NT) xlo[b] = (uint32_t)region_xlo((uint64_t)c * F + b, tv.R);
    for (uint32_t b = tid; b < F; b += NT) scatter_seg_init(l, b, o.start(b));
    __syncthreads();
    block_excl_scan_lds<NT>(pre, pre, nseg + 1);  // in place; pre[nseg] = total
    const uint32_t total = pre[nseg];
    // segment cursor of this thread (its indices grow monotonically): segment cs holds
    // [cb, nb) of the virtual run, both bounds kept in registers
    uint32_t cs = 0, cb = 0, nb = nseg ? pre[1] : 0;
    // two-word keys: level 1 read as / level 2 written as 12-byte records (PartBufs.rec12)
    const bool rin = W == 2 && (pb.rec12 & R12_IN), rout = W == 2 && (pb.rec12 & R12_OUT);
    const uint32_t x0c = rin ? (uint32_t)region_xlo((uint64_t)c * F, tv.R) : 0;  // coarse bin c's lowest x
    const uint64_t* sp = pb.keys1 + seg0 * pb.cap1 * IS;  // segment cs
    // a wave takes 64 * RUNW consecutive positions of the tile (the cursor rarely moves)
    const uint32_t wpos = (uint32_t)(tid >> 6) * (64 * RUNW) + (tid & 63);
    // Every lane loads (past the total: the first key again) and the select is on the address,
    // never on loaded data, so nothing waits for these loads before the tile's ranks use them
    // (a select on the data made every prefetch wait at once: 47 % of the level-2 cycles).
    auto load_tile = [&](uint32_t t0, uint64_t (&tk)[RUNW][W], bool (&ok)[RUNW]) {
#pragma unroll
        for (int q = 0; q < RUNW; q++) {
            const uint32_t i = t0 + wpos + q * 64;
            ok[q] = i < total;
            const uint64_t* src = sp;  // (past the total: the current segment's first item)
            uint64_t item = (seg0 + cs) * pb.cap1;
            if (ok[q]) {
                if (nb <= i) {
                    do {
                        cs++;
                        cb = nb;
                        nb = pre[cs + 1];
                    } while (nb <= i);
                    sp = pb.keys1 + (seg0 + cs) * pb.cap1 * IS;
                }
                src = sp + (uint64_t)(i - cb) * IS;
                item = (seg0 + cs) * pb.cap1 + (i - cb);
            }
            if constexpr (W == 2) {
                // one 16-byte load for either format at the format's byte offset, into the same
                // registers (a 12-byte record is kept raw, decoded when the tile is scattered; its
                // load reads 4 bytes of the next, inside buffers of 16 bytes per item).  Loads into
                // format-specific registers left a copy after each, and the copy made every load
                // wait for all the tile's earlier ones (s_waitcnt vmcnt(0)): 8 serialised latencies
                // per tile
                const uint64_t off = rin ? item * 12 : item * (8 * IS);
                uint32_t v[4];
                __builtin_memcpy(v, reinterpret_cast<const uint8_t*>(pb.keys1) + off, 16);
                tk[q][0] = v[0] | (uint64_t)v[1] << 32;
                tk[q][1] = v[2] | (uint64_t)v[3] << 32;
                (void)src;
                continue;
            }
#pragma unroll
            for (int w = 0; w < W; w++) tk[q][w] = ks_load(src + w);
        }
    };
    uint64_t tk[RUNW][W];
    bool ok[RUNW];
    if (total) load_tile(0, tk, ok);
    for (uint32_t t0 = 0; t0 < total; t0 += TW) {
        // the next tile is loaded into the same registers as soon as this tile's keys sit
        // in LDS, so its loads overlap this tile's write-out (barriers wait for LDS only)
        const bool more = t0 + TW < total;
        auto mid = [&]() {
            if (more) load_tile(t0 + TW, tk, ok);
        };
        if constexpr (W == 2) {
            if (rin) {  // the level-1 records of coarse bin c
                const Rec12 r1{pb.r12_hb, pb.r12_xb1};
#pragma unroll
                for (int q = 0; q < RUNW; q++) {
                    const uint3 v = make_uint3((uint32_t)tk[q][0], (uint32_t)(tk[q][0] >> 32), (uint32_t)tk[q][1]);
                    r1.dec(v, x0c, tk[q][0], tk[q][1]);
                }
            }
        }
        if constexpr (REC6) {
            scatter_seg<W, RUNW, BinRegion, OutSeg, NT>(l, F, bin, o, tk, ok, pb.keys2, mid,
                                                        StoreRec6{xlo});
        } else if constexpr (W == 2) {
            scatter_seg<W, RUNW, BinRegion, OutSeg, NT>(l, F, bin, o, tk, ok, pb.keys2, mid,
                                                        StoreW2{rout, Rec12{pb.r12_hb, pb.r12_xb2}});
        } else {
            scatter_seg<W, RUNW, BinRegion, OutSeg, NT>(l, F, bin, o, tk, ok, pb.keys2, mid);
        }
    }
    __syncthreads();  // the last write-out read lim / gbase
    for (uint32_t b = tid; b < F; b += NT)
        pb.hist2[((uint64_t)c * F + b) * B2T + jo] = (uint32_t)(scatter_seg_next(l, b) - o.start(b));
}

// LDS image of a region: the 16-byte chunks of each 128-byte bucket are XOR-swizzled
// with the bucket index so that lanes probing random buckets spread over the banks.
// (bits 1..3 of the bucket: with bit 0 selecting the 128-byte half of a 256-byte bank row,
// the chunk of a random bucket lands on any of the 16 bank quads)
DEV uint32_t lds_chunk(uint32_t b, uint32_t q) { return b * 8 + (q ^ ((b >> 1) & 7)); }
DEV uint64_t* lds_word(uint64_t* lt, uint32_t b, uint32_t word) {
    return lt + lds_chunk(b, word >> 1) * 2 + (word & 1);
}

// 8-bit slot tags (LDS only, beside the region image): one u64 per bucket, byte s = the tag
// of slot s, 0 = empty.  A probe reads the bucket's tags (one ds_read_b64) and the key words
// of the slots whose tag matches, instead of every key word of the bucket.
DEV uint32_t slot_tag(uint64_t t0) { return 1u + (((uint32_t)t0 & 0xFFu) * 255u >> 8); }
// bit i set iff byte i of x is zero (exact: no borrow between bytes)
DEV uint32_t zero_byte_mask4(uint32_t x) {
    const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);  // bit 7 of each zero byte
    return ((z >> 7) * 0x01020408u) >> 24;                                       // bits 7/15/23/31 -> 0..3
}
DEV uint32_t zero_byte_mask8(uint64_t x) {
    return zero_byte_mask4((uint32_t)x) | zero_byte_mask4((uint32_t)(x >> 32)) << 4;
}

// Exclusive prefix of a level-3 workgroup's n <= MAX_SEG_GROUP segment fills (s_pre[0..n],
// s_pre[n] = total), by the first wave: two fills per lane, one DPP scan (was a one-thread loop
// of n dependent-looking loads, ~n HBM latencies at every workgroup's start)
// s_pp (if given): the same prefix of the fills' record pairs, ceil(fill / 2) (k_p3's 6-byte records)
DEV void seg_prefix(uint32_t* s_pre, const uint32_t* __restrict__ fill, uint32_t n, uint32_t* s_pp = nullptr) {
    if (threadIdx.x < 64) {
        const uint32_t j = 2 * threadIdx.x;
        const uint32_t a = j < n ? fill[j] : 0, b = j + 1 < n ? fill[j + 1] : 0;
        const uint32_t inc = wave_incl_sum(a + b);
        const uint32_t ex = inc - (a + b);
        if (j < n) s_pre[j] = ex;
        if (j + 1 < n) s_pre[j + 1] = ex + a;
        if (threadIdx.x == 63) s_pre[n] = inc;
        if (s_pp) {
            const uint32_t pa = (a + 1) >> 1, pb = (b + 1) >> 1;
            const uint32_t pinc = wave_incl_sum(pa + pb);
            const uint32_t pex = pinc - (pa + pb);
            if (j < n) s_pp[j] = pex;
            if (j + 1 < n) s_pp[j + 1] = pex + pa;
            if (threadIdx.x == 63) s_pp[n] = pinc;
        }
    }
}

// Level 3: one workgroup per region: LDS-resident table
// SEG: the region's keys are the B2 level-2 segments (region, j) (fills in hist2);
// otherwise the contiguous run [off2[r * B2], off2[(r + 1) * B2]).  A segmented launch
// leaves the table alone when the batch overflowed; an exact one can be gated.
// CNT: items are {W key words, count} records (shard merge) and add their count.
// fresh: the table is known to be all zero (just reset), so the region is not read.
// GATE: Bloom pass 2 on the blocked layout: an item is inserted only if its filter-2 bits
// are set (parallel_parser.hpp:2436-2441).  The blocks of a region's keys form one
// contiguous slice of the filter (bloom_block and region_of share the hash prefix), so
// the gate reads stay within a few KiB that L2 keeps.
constexpr int P3_THREADS = 1024;  // two 64 KiB regions per CU: 8 waves per SIMD

// REC6: the segments hold 6-byte level-2 records (StoreRec6; one-word keys, SEG, not CNT)
template <int W, bool SEG, bool CNT, bool GATE = false, bool REC6 = false>
__global__ __launch_bounds__(P3_THREADS, P3_THREADS / 128) void k_p3(TableView tv, PartBufs pb,
                                                                  DevCounters* __restrict__ ctr,
                                                                  const unsigned long long* gate, int fresh,
                                                                  BloomView bf) {
    constexpr int NT = P3_THREADS;
    constexpr int IW = CNT ? W + 1 : W;  // words per item
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint32_t s_pre[MAX_SEG_GROUP + 1];  // SEG: exclusive prefix of the B2 segment fills
    __shared__ uint32_t s_pp[REC6 ? MAX_SEG_GROUP + 1 : 1];  // REC6: ... of their record pairs
    constexpr int S = BUCKET_WORDS / (W + 1);
    // keys loaded per thread before inserting (memory-level parallelism); 1024-thread
    // groups already keep 8 waves per SIMD in flight
    // (8 one-word keys measured 1 % faster but spill; 3-4 two-word keys no faster: r02_v22/v23)
    constexpr int KB = NT >= 1024 ? (CNT || W > 1 ? 2 : 4) : 8;  // (CNT items carry a count: 64 VGPRs)
    if constexpr (SEG) {
        if (ctr->part_overflow) return;
    } else {
        if (gated_off(gate)) return;
    }
    uint64_t* lt = reinterpret_cast<uint64_t*>(smem);  // BPR * BUCKET_WORDS words
    uint64_t* tg = lt + BPR * BUCKET_WORDS;             // BPR tag words (slot_tag of each slot's word 0)
    const uint64_t r = blockIdx.x;
    uint64_t start, end;
    // runs (the merge over region-sorted groups): each group's first record in LDS, so an item's
    // address needs no dependent global load
    // (runs are count records: the other variants keep their static LDS, which the gate's filter
    // slice budget counts on)
    __shared__ uint64_t s_gst[SEG && CNT ? MAX_SEG_GROUP : 1];
    if constexpr (SEG) {
        seg_prefix(s_pre, pb.hist2 + r * pb.B2, pb.B2, REC6 ? s_pp : nullptr);
        if constexpr (CNT)
            if (pb.seg_start)
                for (uint32_t g = threadIdx.x; g < pb.B2; g += NT) s_gst[g] = pb.seg_start[r * pb.B2 + g];
        __syncthreads();
        start = 0;
        end = __builtin_amdgcn_readfirstlane(s_pre[pb.B2]);  // (uniform: the round loop's branches are scalar)
    } else {
        start = pb.off2[r * pb.B2];
        end = pb.off2[(r + 1) * pb.B2];
    }
    // nothing to insert: leave the region untouched, unless the table is fresh (its reset may
    // have been deferred to this pass, which then writes every region)
    if (start == end && !fresh) return;
    uint4* g4 = reinterpret_cast<uint4*>(tv.buckets + r * BPR * BUCKET_WORDS);
    uint4* l4 = reinterpret_cast<uint4*>(lt);
    constexpr int N4 = BPR * BUCKET_WORDS / 2;
    constexpr int NT4 = BPR / 2;  // tag words, as uint4
    if (fresh) {
        for (int i = threadIdx.x; i < N4 + NT4; i += NT) l4[i] = make_uint4(0, 0, 0, 0);
        __syncthreads();
    } else {
        for (int i = threadIdx.x; i < N4; i += NT) l4[lds_chunk(i >> 3, i & 7)] = g4[i];
        __syncthreads();
        {
            for (int bb = threadIdx.x; bb < BPR; bb += NT) {
                uint64_t t = 0;
#pragma unroll
                for (int sl = 0; sl < S; sl++) {
                    const uint64_t w0 = *lds_word(lt, bb, sl * W);
                    if (w0 != EMPTY) t |= (uint64_t)slot_tag(w0) << (8 * sl);
                }
                tg[bb] = t;
            }
            __syncthreads();
        }
    }
    // GATE with an LDS slice: the filter-2 bits of the region's blocks, 8 words per block
    uint32_t* gs = reinterpret_cast<uint32_t*>(tg + BPR);
    uint64_t gblo = 0;
    if constexpr (GATE) {
        if (bf.slice_blocks) {
            uint64_t ghi;
            region_blocks(r, tv.R, bf.nblocks, gblo, ghi);
            const uint32_t n4 = (uint32_t)(ghi - gblo + 1) * 2;  // filter-2 halves of the blocks, as uint4
            const uint4* src = reinterpret_cast<const uint4*>(bf.bits + gblo * BF_BLOCK_WORDS);
            uint4* dst = reinterpret_cast<uint4*>(gs);
            for (uint32_t i = threadIdx.x; i < n4; i += NT) dst[i] = src[(i >> 1) * 4 + 2 + (i & 1)];
            __syncthreads();
        }
    }
    uint32_t n_fail = 0, n_ins = 0;
    unsigned long long n_add = 0;  // CNT: the records' counts (the runs merge counts them here)
    // SEG: segment cursor of this thread (indices grow monotonically): segment cs holds
    // [cb, nb), both bounds in registers
    uint32_t cs = 0, cb = 0, nb = 0;
    if constexpr (SEG) nb = s_pre[1];
    // Runs (the merge over region-sorted groups): a sender's records sit in its table order,
    // i.e. sorted by home bucket, and inserted in that order neighbouring lanes collide on
    // the same buckets and banks.  The items are visited in a scrambled order instead: a
    // bijection of [0, 2^m) (2^m >= end), slots mapping past end are idle.
    const bool runs = SEG && pb.seg_start != nullptr;
    uint64_t vend = end;
    uint32_t pmask = 0, psh = 0;
    if (runs && end > 1) {
        const uint32_t m = 64 - __builtin_clzll(end - 1);
        vend = 1ULL << m;
        pmask = (uint32_t)(vend - 1);
        psh = (m + 1) / 2;
    }
    static_assert(!REC6 || (W == 1 && SEG && !CNT), "6-byte records: one-word keys in segments");
    const bool r12 = W == 2 && SEG && !CNT && (pb.rec12 & R12_L2);  // Rec12 level-2 records
    // (in the table's geometry, R12_REG: decoded against region r's lowest x; from the Bloom
    // pass's fine bins: against the fine bin's)
    const bool r12_reg = r12 && (pb.rec12 & R12_REG);
    const uint32_t xlo_r = REC6 || r12_reg ? (uint32_t)region_xlo(r, tv.R) : 0;
    // sg: Rec12 items' fine bin (seg >> r12_b2s), beside the raw record
    auto load_items = [&](uint64_t base, uint64_t (&kk)[KB][W], uint64_t (&add)[KB], uint32_t& ok,
                          uint32_t (&sg)[KB]) {
        ok = 0;
#pragma unroll
        for (int q = 0; q < KB; q++) {
            const uint64_t i = base + threadIdx.x + (uint64_t)q * NT;
            if constexpr (W == 2 && SEG && !CNT) {
                // either format (a 12-byte record, kept raw with its fine bin and decoded when
                // used, or two whole words) by one 16-byte load into the same registers, at the
                // format's byte offset (k_p2f load_tile: format-specific registers made every load
                // wait for the earlier ones); lanes past the end load their segment's first item
                uint64_t seg = r * pb.B2 + cs, item = seg * pb.cap2;
                if (i < end) {
                    while (nb <= i) {
                        cs++;
                        cb = nb;
                        nb = s_pre[cs + 1];
                    }
                    seg = r * pb.B2 + cs;
                    item = seg * pb.cap2 + (i - cb);
                    ok |= 1u << q;
                }
                uint32_t v[4];
                __builtin_memcpy(v, reinterpret_cast<const uint8_t*>(pb.keys2) + (r12 ? item * 12 : item * 16), 16);
                kk[q][0] = v[0] | (uint64_t)v[1] << 32;
                kk[q][1] = v[2] | (uint64_t)v[3] << 32;
                sg[q] = (uint32_t)(seg >> pb.r12_b2s);
                add[q] = 1;
                continue;
            }
            // every lane loads (past the end: a nearby item) into the same registers, its validity in
            // ok and its count masked where it is used: a value merged after a load made every
            // load wait for the earlier ones
            const uint64_t* src = nullptr;
            if (runs) {
                uint32_t j = ((uint32_t)i * 0x9E3779B1u) & pmask;
                j ^= j >> psh;
                j = (j * 0x85EBCA77u) & pmask;
                if (i < vend && j < end) {
                    uint32_t lo = 0, hi = pb.B2;  // the group holding j: s_pre[lo] <= j < s_pre[lo + 1]
                    while (hi - lo > 1) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (s_pre[mid] <= j) lo = mid;
                        else hi = mid;
                    }
                    src = pb.keys2 + ((CNT ? s_gst[lo] : pb.seg_start[r * pb.B2 + lo]) + (j - s_pre[lo])) * IW;
                }
            } else if (i < end) {
                if constexpr (SEG) {
                    while (nb <= i) {
                        cs++;
                        cb = nb;
                        nb = s_pre[cs + 1];
                    }
                    src = pb.keys2 + ((r * pb.B2 + cs) * pb.cap2 + (i - cb)) * IW;
                } else {
                    src = pb.keys2 + i * IW;
                }
            }
            ok |= (src != nullptr) << q;
            if (!src) src = pb.keys2 + (SEG ? (r * pb.B2 + cs) * pb.cap2 * IW : start * IW);  // (a nearby item)
#pragma unroll
            for (int w = 0; w < W; w++) kk[q][w] = ks_load(src + w);
            if constexpr (CNT) add[q] = src[W];  // (raw: CNT_MASK applied where it is used)
            else add[q] = 1;
        }
    };

    // one key into the LDS region (tag probe, claim by CAS on word 0, count add); false: the
    // region's probe bound was reached (counted as an overflow)
    auto insert_one = [&](const uint64_t (&kw)[W], uint64_t a0) -> bool {
        const uint64_t k0 = kw[0];
        uint32_t b = bucket_in_region(k0, tv.R);
        bool done = false;
        {
            constexpr uint32_t SMASK = (1u << S) - 1;
            const uint32_t tag = slot_tag(k0);
            const uint64_t bc = 0x0101010101010101ULL * tag;
            for (int probe = 0; probe < 4 * BPR && !done;) {
                const uint64_t tw = tg[b];
                uint32_t m = zero_byte_mask8(tw ^ bc) & SMASK;
                int slot = -1;
                while (m) {  // candidates: usually none (new key) or exactly the key's slot
                    const int sl = __builtin_ctz(m);
                    m &= m - 1;
                    bool eq = *lds_word(lt, b, sl * W) == k0;
#pragma unroll
                    for (int w = 1; w < W; w++) eq &= *lds_word(lt, b, sl * W + w) == kw[w];
                    if (eq) {
                        slot = sl;
                        break;
                    }
                }
                uint64_t a = a0;
                if (slot < 0) {
                    const uint32_t em = zero_byte_mask8(tw) & SMASK;
                    if (!em) {  // bucket full, key absent: next bucket
                        b = (b + 1) & (BPR - 1);
                        probe++;
                        continue;
                    }
                    // claim the first untagged slot by its word 0; the tag is stored last, so
                    // a tag match always finds the key's words published
                    const int e = __builtin_ctz(em);
                    const uint64_t old = atomicCAS(reinterpret_cast<unsigned long long*>(lds_word(lt, b, e * W)),
                                                   0ULL, (unsigned long long)k0);
                    if (old == EMPTY) {
#pragma unroll
                        for (int w = 1; w < W; w++)
                            __hip_atomic_store(lds_word(lt, b, e * W + w), kw[w], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        __hip_atomic_store(reinterpret_cast<uint8_t*>(tg + b) + e, (uint8_t)tag, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                        if constexpr (W > 1) a += READY;  // the table format's published flag
                        slot = e;
                    } else if (W == 1 && old == k0) {
                        slot = e;  // the same key, claimed an instant ago
                    } else {
                        probe++;  // claimed by another key (tag not yet stored): read again
                        continue;
                    }
                }
                atomicAdd(reinterpret_cast<unsigned long long*>(lds_word(lt, b, S * W + slot)),
                          (unsigned long long)a);
                done = true;
            }
        }

        return done;
    };

    if constexpr (REC6) {
        // 6-byte records by pairs: one 12-byte load gives two keys (the pair's three dwords
        // {lo_even, lo_odd, d_even | d_odd << 16}, StoreRec6), KP pairs per thread and round with
        // the next round's loads issued first: half the loads and rounds of one record per load.
        // s_pp: exclusive prefix of the segments' pair counts; the last pair of an odd fill
        // holds one record
        constexpr int KP = GATE ? 2 : 4;  // (the gate's filter words: 4 pairs spill)
        const uint32_t endp = __builtin_amdgcn_readfirstlane(s_pp[pb.B2]);  // (uniform: scalar branches)
        uint32_t ps = 0, pcb = 0, pnb = s_pp[1], pfill = s_pre[1];
        auto load_pairs = [&](uint32_t base, uint3 (&v)[KP], uint32_t& ok) {
            // the pairs' addresses first (the segment cursor's loop), then every load back to back
            uint64_t pp[KP];
            ok = 0;
#pragma unroll
            for (int q = 0; q < KP; q++) {
                const uint32_t j = base + threadIdx.x + (uint32_t)q * NT;
                pp[q] = 0;
                if (j < endp) {  // (loads only in range, as the one-record form)
                    while (pnb <= j) {
                        ps++;
                        pcb = pnb;
                        pnb = s_pp[ps + 1];
                        pfill = s_pre[ps + 1] - s_pre[ps];
                    }
                    pp[q] = ((r * pb.B2 + ps) * pb.cap2 >> 1) + (j - pcb);
                    ok |= (1u | (uint32_t)(2 * (j - pcb) + 1 < pfill) << 1) << (2 * q);
                }
            }
            // (every slot loads, a slot without a pair the buffer's first: a load under a branch
            // was waited for inside it, where its registers merge with the other path's)
#pragma unroll
            for (int q = 0; q < KP; q++) {
                uint32_t w3[3];
                __builtin_memcpy(w3, reinterpret_cast<const uint32_t*>(pb.keys2) + pp[q] * 3, 12);
                v[q] = make_uint3(w3[0], w3[1], w3[2]);
            }
        };
        uint3 cv[KP];
        uint32_t cok = 0;
        if (endp) load_pairs(0, cv, cok);
        for (uint32_t base = 0; base < endp; base += (uint32_t)KP * NT) {
            uint3 nv[KP];
            uint32_t nok = 0;
            // (the next round's loads unconditionally: past the end every slot reads the buffer's
            // first pair, ok = 0; under a branch the loads were waited for as soon as issued)
            load_pairs(base + (uint32_t)KP * NT, nv, nok);
            uint64_t kp[2 * KP][1];
            bool pass[2 * KP];
#pragma unroll
            for (int q = 0; q < KP; q++) {
                kp[2 * q][0] = ((uint64_t)(xlo_r + (cv[q].z & 0xFFFFu)) << 32) | cv[q].x;
                kp[2 * q + 1][0] = ((uint64_t)(xlo_r + (cv[q].z >> 16)) << 32) | cv[q].y;
            }
#pragma unroll
            for (int q = 0; q < 2 * KP; q++) {  // the gate reads of all items are issued together
                pass[q] = (cok >> q) & 1;
                if constexpr (GATE) {
                    const uint64_t t0 = kp[q][0];
                    if (bf.slice_blocks)
                        pass[q] = pass[q] && block_gate(gs + (bloom_block(t0, bf.nblocks) - gblo) * 8, t0, bf.nh_gate);
                    else
                        pass[q] = pass[q] && block_gate(bloom_block_ptr(bf, t0) + 8, t0, bf.nh_gate);
                }
                n_ins += pass[q];
            }
#pragma unroll
            for (int q = 0; q < 2 * KP; q++)
                if (pass[q] && !insert_one(kp[q], 1)) n_fail++;
#pragma unroll
            for (int q = 0; q < KP; q++) cv[q] = nv[q];
            cok = nok;
        }
    } else {
        struct Items {
            uint64_t kk[KB][W];
            uint64_t add[KB];
            uint32_t okm, sg[KB];
        };
        // one round of KB items per thread: decode, gate, insert
        auto round = [&](Items& it) {
            if constexpr (W == 2) {
                if (r12) {
                    const Rec12 rc{pb.r12_hb, pb.r12_xb2};
#pragma unroll
                    for (int q = 0; q < KB; q++) {
                        const uint3 v = make_uint3((uint32_t)it.kk[q][0], (uint32_t)(it.kk[q][0] >> 32), (uint32_t)it.kk[q][1]);
                        rc.dec(v, r12_reg ? xlo_r : it.sg[q] << pb.r12_xb2, it.kk[q][0], it.kk[q][1]);
                    }
                }
            }
            bool pass[KB];
#pragma unroll
            for (int q = 0; q < KB; q++) {  // the gate reads of all KB items are issued together
                pass[q] = (it.okm >> q) & 1;
                if constexpr (GATE) {
                    const uint64_t t0 = it.kk[q][0];
                    if (bf.slice_blocks)
                        pass[q] = pass[q] && block_gate(gs + (bloom_block(t0, bf.nblocks) - gblo) * 8, t0, bf.nh_gate);
                    else
                        pass[q] = pass[q] && block_gate(bloom_block_ptr(bf, t0) + 8, t0, bf.nh_gate);
                }
                n_ins += pass[q];
                if constexpr (CNT) {
                    it.add[q] &= CNT_MASK;
                    n_add += pass[q] ? it.add[q] : 0;
                }
            }
#pragma unroll
            for (int q = 0; q < KB; q++)
                if (pass[q] && !insert_one(it.kk[q], it.add[q])) n_fail++;
        };
        constexpr uint64_t STEP = (uint64_t)KB * NT;
        if constexpr (W <= 2) {
            // ping-pong rounds: the next round's items load into the other buffer while this one is
            // inserted (unconditionally: past the end a slot reads a nearby item, ok = 0).  Copying
            // the prefetched items into the current buffer at each round's end made the compiler
            // wait for the prefetch right after issuing it
            Items ia, ib;
            load_items(start, ia.kk, ia.add, ia.okm, ia.sg);
            for (uint64_t base = start; base < vend; base += 2 * STEP) {
                load_items(base + STEP, ib.kk, ib.add, ib.okm, ib.sg);
                round(ia);
                if (base + STEP >= vend) break;
                load_items(base + 2 * STEP, ia.kk, ia.add, ia.okm, ia.sg);
                round(ib);
            }
        } else {  // (W > 2: no spare registers for a second buffer)
            Items ia;
            for (uint64_t base = start; base < vend; base += STEP) {
                load_items(base, ia.kk, ia.add, ia.okm, ia.sg);
                round(ia);
            }
        }
    }
    __syncthreads();
    // kc_route_hint: the region's records per owner shard for each of its two 256-bucket route
    // blocks, counted in s_pre (dead once the items are inserted)
    const uint32_t op = pb.own_parts;
    static_assert(MAX_SEG_GROUP + 1 >= 2 * RT_MAX_PARTS && BPR == 512, "owner counters in s_pre, two route blocks");
    if (op)
        for (uint32_t i = threadIdx.x; i < 2 * RT_MAX_PARTS; i += NT) s_pre[i] = 0;
    for (int i = threadIdx.x; i < N4; i += NT) g4[i] = l4[lds_chunk(i >> 3, i & 7)];
    if (op) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < BPR * S; i += NT) {
            const uint32_t bb = i / S, sl = i % S;
            const uint64_t w0 = *lds_word(lt, bb, sl * W);
            if (w0 != EMPTY) atomicAdd(&s_pre[(bb >= BPR / 2 ? RT_MAX_PARTS : 0) + owner_of(w0, op)], 1u);
        }
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < 2 * op; i += NT) {
            const uint32_t h = i / op, d = i % op;
            pb.own_hist[(uint64_t)d * pb.own_nblk + 2 * r + h] = s_pre[h * RT_MAX_PARTS + d];
        }
    }
    if (n_fail) atomicAdd(&ctr->overflow, (unsigned long long)n_fail);
    if constexpr (GATE || CNT) {
        // GATE: the gated insertions (level 1 counted the windows); CNT over runs: the
        // records' counts (the general merge insert counted them at its level 1).  One
        // atomic per workgroup: per-wave adds to this one counter from every region's
        // workgroup serialise at the memory-side atomic unit (milliseconds per pass)
        block_add4(GATE ? (CNT ? n_add : n_ins) : (pb.seg_start ? n_add : 0), 0, 0, 0, &ctr->inserted, nullptr, nullptr,
                   nullptr);
    }
}

// Bloom pass 1, level 3 (blocked layout): one workgroup per filter region of `bpr`
// blocks (64 KiB): the region -> LDS (zero-filled when the filter is fresh), the
// reference's insertion_process for every key of the region with LDS atomics
// (block_insert), the region back to HBM.  Replaces one scattered device-scope atomic per
// bit (the direct pass) with two sequential sweeps of the filter per batch.
// SEG: the region's keys are its B2 level-2 segments (fills in hist2); otherwise the
// contiguous run [off2[r * B2], off2[(r + 1) * B2]).
// keys per thread per round and workgroup size: 512 threads keep the insertion path within
// its registers (72 VGPRs, no scratch spills; 1024-thread groups would be capped at 64)
constexpr int B3_THREADS = 512;  // two 64 KiB regions per CU
template <bool SEG>
__global__ __launch_bounds__(B3_THREADS, B3_THREADS / 128) void k_b3(BloomView bf, uint32_t bpr, PartBufs pb,
                                                                  DevCounters* __restrict__ ctr,
                                                                  const unsigned long long* gate, int fresh, int is,
                                                                  int cntw, int rec_phase) {
    // is: u64 words per item (word 0 is the table key word the filter uses); cntw >= 0: items
    // are pre-aggregated {key, count} records (kc_bloom_records_device) with the count in word
    // cntw, and a record of count >= 2 takes insertion_process twice -- the filter updates of a
    // k-mer seen twice, as the reference makes them (double_bloomfilter.hpp:371-413).  The
    // records are distinct keys; rec_phase 0 inserts those of count >= 2, rec_phase 1 (a later
    // launch) those of count 1, with the distinct-key rule of block_insert: the order "the
    // k-mers seen twice first", one sequential order of the reference's pass
    constexpr int NT = B3_THREADS, KB = 4;  // (8 or 2 keys per round: slower, r02_v21)
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint32_t s_pre[MAX_SEG_GROUP + 1];
    if constexpr (SEG) {
        if (ctr->part_overflow) return;
    } else {
        if (gated_off(gate)) return;
    }
    uint32_t* lf = reinterpret_cast<uint32_t*>(smem);
    const uint64_t r = blockIdx.x;
    uint64_t start, end;
    if constexpr (SEG) {
        seg_prefix(s_pre, pb.hist2 + r * pb.B2, pb.B2);
        __syncthreads();
        start = 0;
        end = __builtin_amdgcn_readfirstlane(s_pre[pb.B2]);  // (uniform: the round loop's branches are scalar)
    } else {
        start = pb.off2[r * pb.B2];
        end = pb.off2[(r + 1) * pb.B2];
    }
    if (start == end) return;  // the region keeps its bits (a fresh filter is zero already)
    const uint32_t n4 = bpr * BF_BLOCK_WORDS / 4;
    uint4* g4 = reinterpret_cast<uint4*>(bf.bits + r * bpr * BF_BLOCK_WORDS);
    uint4* l4 = reinterpret_cast<uint4*>(lf);
    for (uint32_t i = threadIdx.x; i < n4; i += NT) l4[i] = fresh ? make_uint4(0, 0, 0, 0) : g4[i];
    __syncthreads();
    const uint64_t blk0 = r * bpr;
    const int lane = threadIdx.x & 63;
    uint64_t* wq = reinterpret_cast<uint64_t*>(smem + (size_t)bpr * BF_BLOCK_WORDS * 4) + (threadIdx.x >> 6) * 64;
    uint32_t* wf = reinterpret_cast<uint32_t*>(smem + (size_t)bpr * BF_BLOCK_WORDS * 4 + (size_t)(NT / 64) * 64 * 8) +
                   (threadIdx.x >> 6) * 64;  // (cntw >= 0: the queue entries' counts >= 2)
    BloomLocal bl = {0, 0, 0};
    uint32_t cs = 0, cb = 0, nb = 0;  // SEG: segment cursor (indices grow monotonically)
    if constexpr (SEG) nb = s_pre[1];
    const bool r12 = SEG && (pb.rec12 & R12_L2);  // 12-byte records of fine bin seg >> r12_b2s (Rec12)
    // the next round's items are loaded while this round's are tested and inserted (the loads'
    // latency was exposed once per round; raw records, decoded when used)
    struct Raw {
        uint3 v[KB];
        uint32_t xhi[KB];
        uint64_t cnt[KB];  // cntw >= 0: the records' count words
    };
    auto fetch = [&](uint64_t base, Raw& w) {
#pragma unroll
        for (int q = 0; q < KB; q++) {
            const uint64_t i = base + threadIdx.x + (uint64_t)q * NT;
            if constexpr (SEG) {
                // either format by one 12-byte load into the same registers at the format's byte
                // offset (k_p2f load_tile: format-specific registers made every load wait for the
                // earlier ones); lanes past the end load their segment's first item, a whole word's load reads 4 bytes
                // of the next item (z, unused)
                uint64_t seg = r * pb.B2 + cs, item = seg * pb.cap2;  // (past the end: the segment's first)
                if (i < end) {
                    while (nb <= i) {
                        cs++;
                        cb = nb;
                        nb = s_pre[cs + 1];
                    }
                    seg = r * pb.B2 + cs;
                    item = seg * pb.cap2 + (i - cb);
                }
                uint32_t v[3];
                __builtin_memcpy(v, reinterpret_cast<const uint8_t*>(pb.keys2) + (r12 ? item * 12 : item * is * 8), 12);
                w.v[q] = make_uint3(v[0], v[1], v[2]);
                w.xhi[q] = r12 ? (uint32_t)(seg >> pb.r12_b2s) << pb.r12_xb2 : 0;
                continue;
            }
            // the contiguous run (exact layout, or {key, count} records): the count word raw, its
            // phase test made when the round uses it (a test here would wait for the load)
            const uint64_t ii = i < end ? i : 0;
            const uint64_t t = pb.keys2[ii * is];
            w.v[q] = make_uint3((uint32_t)t, (uint32_t)(t >> 32), 0);
            w.xhi[q] = 0;
            w.cnt[q] = cntw >= 0 ? pb.keys2[ii * is + cntw] : 0;
        }
    };
    // one round: KB items per thread, the fast path, then the wave's queue of slow items
    auto round = [&](const Raw& cur, uint64_t base) {
    uint64_t t0[KB];
        uint32_t two = 0;  // bit q: item q is a record of count >= 2
#pragma unroll
        for (int q = 0; q < KB; q++) {
            t0[q] = r12 ? (uint64_t)(cur.xhi[q] | cur.v[q].z >> (pb.r12_hb + 1)) << 32 | cur.v[q].x
                        : (uint64_t)cur.v[q].y << 32 | cur.v[q].x;
            if (cntw >= 0) {
                const bool tw = (cur.cnt[q] & CNT_MASK) >= 2;
                two |= (uint32_t)tw << q;
                if (tw != (rec_phase == 0)) t0[q] = EMPTY;  // (the other phase's: skipped)
            }
        }
        // fast path: a k-mer whose filter-2 bits are all set changes nothing (most
        // occurrences of a k-mer seen before); the others are packed into the wave's queue
        // so the insertion path runs on dense lanes instead of once per item slot
        bool slow[KB];
        uint32_t pre[KB], rank[KB], total = 0;
#pragma unroll
        for (int q = 0; q < KB; q++) {
            // (every slot reads its block, clamped into the region: no read under a branch, so
            // the KB gate reads wait once together)
            const uint32_t lb = (uint32_t)min(bloom_block(t0[q], bf.nblocks) - blk0, (uint64_t)bpr - 1);
            slow[q] = !block_gate(lf + lb * BF_BLOCK_WORDS + 8, t0[q], bf.nh) &&
                      base + threadIdx.x + (uint64_t)q * NT < end && (cntw < 0 || t0[q] != EMPTY);
        }
#pragma unroll
        for (int q = 0; q < KB; q++) {  // (the ballots after all the gate reads)
            const uint64_t bal = __ballot(slow[q]);
            pre[q] = total;
            rank[q] = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
            total += (uint32_t)__popcll(bal);
        }
        for (uint32_t r0 = 0; r0 < total; r0 += 64) {
#pragma unroll
            for (int q = 0; q < KB; q++)
                if (slow[q] && pre[q] + rank[q] - r0 < 64) {
                    wq[pre[q] + rank[q] - r0] = t0[q];
                    if (cntw >= 0) wf[pre[q] + rank[q] - r0] = (two >> q) & 1;
                }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's queue writes land
            if (lane < total - r0) {
                const uint64_t t = wq[lane];
                const uint32_t lb = (uint32_t)(bloom_block(t, bf.nblocks) - blk0);
                block_insert(lf + lb * BF_BLOCK_WORDS, t, bf.nh, bl, cntw >= 0);
                if (cntw >= 0 && wf[lane]) block_insert(lf + lb * BF_BLOCK_WORDS, t, bf.nh, bl, true);  // its second sighting
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // queue reads done before reuse
        }
    };
    // ping-pong rounds: the next round's items load into the other buffer while this one is
    // processed (unconditionally: past the end a slot reads a nearby item and is not used).  A
    // copy of the prefetched buffer into the current one at each round's end made the compiler
    // wait for the prefetch right after issuing it
    constexpr uint64_t STEP = (uint64_t)KB * NT;
    Raw ra, rb;
    fetch(start, ra);
    for (uint64_t base = start; base < end; base += 2 * STEP) {
        fetch(base + STEP, rb);
        round(ra, base);
        if (base + STEP >= end) break;
        fetch(base + 2 * STEP, ra);
        round(rb, base + STEP);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n4; i += NT) g4[i] = l4[i];
    // one atomic per counter and workgroup (per-wave adds to one address serialise)
    block_add4(bl.new_first, bl.new_second, bl.failed, 0, &ctr->new_in_first, &ctr->new_in_second,
               &ctr->failed_in_first, nullptr);
}

// --------------------------------------------------------------------------------
// shard merge over region-sorted groups (kc_insert_counts_runs_device): the records a
// rank receives are G groups (one per sender), each in the sender's table order, i.e.
// sorted by region when the sender's table has this table's geometry.  Region run bounds
// per group by binary search, then one level-3 pass (k_p3<W, SEG, CNT> over the runs):
// the partition levels of the general merge insert are not needed.
// --------------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(256) void k_check_runs(const uint64_t* __restrict__ rec, const uint64_t* __restrict__ gstart,
                                                    uint64_t R, unsigned long long* flag) {
    const uint32_t g = blockIdx.y;
    const uint64_t lo = gstart[g], hi = gstart[g + 1];
    bool bad = false;
    for (uint64_t i = lo + 1 + (uint64_t)blockIdx.x * 256 + threadIdx.x; i < hi; i += (uint64_t)gridDim.x * 256)
        bad |= region_of(rec[i * (W + 1)], R) < region_of(rec[(i - 1) * (W + 1)], R);
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1ULL);
}
// m_start[r * G + g] = first record of group g with region >= r (r = 0..R)
template <int W>
__global__ __launch_bounds__(256) void k_run_bounds(const uint64_t* __restrict__ rec,
                                                    const uint64_t* __restrict__ gstart, uint32_t G, uint64_t R,
                                                    uint64_t* __restrict__ m_start) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (R + 1) * G) return;
    const uint64_t r = t / G;
    const uint32_t g = (uint32_t)(t % G);
    uint64_t lo = gstart[g], hi = gstart[g + 1];  // first index in [lo, hi) with region >= r
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (region_of(rec[mid * (W + 1)], R) < r) lo = mid + 1;
        else hi = mid;
    }
    m_start[t] = lo;
}
static __global__ __launch_bounds__(256) void k_run_lengths(const uint64_t* __restrict__ m_start, uint64_t RG, uint32_t G,
                                                     uint32_t* __restrict__ m_len) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t < RG) m_len[t] = (uint32_t)(m_start[t + G] - m_start[t]);
}

// exclusive scan of n u32 -> u64 (out has n+1 entries), three passes:
// per-block scans of 4096 elements, a scan of the block sums, the add-back
constexpr int SCAN_T = 1024;
constexpr int SCAN_PER = 4;
DEV unsigned long long block_incl_sum_1024(unsigned long long v) {
    __shared__ unsigned long long s_w[SCAN_T / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    if (lane == 63) s_w[wid] = v;
    __syncthreads();
    unsigned long long base = 0;
    for (int w = 0; w < wid; w++) base += s_w[w];
    __syncthreads();
    return v + base;
}
static __global__ __launch_bounds__(SCAN_T) void k_scanA(const uint32_t* __restrict__ in, uint64_t n,
                                                 uint64_t* __restrict__ out, uint64_t* __restrict__ bsum,
                                                 const unsigned long long* gate) {
    if (gated_off(gate)) return;
    const uint64_t i0 = ((uint64_t)blockIdx.x * SCAN_T + threadIdx.x) * SCAN_PER;
    uint32_t v[SCAN_PER];
    unsigned long long sum = 0;
#pragma unroll
    for (int q = 0; q < SCAN_PER; q++) {
        v[q] = i0 + q < n ? in[i0 + q] : 0;
        sum += v[q];
    }
    const unsigned long long incl = block_incl_sum_1024(sum);
    unsigned long long run = incl - sum;
#pragma unroll
    for (int q = 0; q < SCAN_PER; q++) {
        if (i0 + q < n) out[i0 + q] = run;
        run += v[q];
    }
    if (threadIdx.x == SCAN_T - 1) bsum[blockIdx.x] = incl;
}
static __global__ __launch_bounds__(SCAN_T) void k_scanB(uint64_t* __restrict__ bsum, uint64_t nb, uint64_t* __restrict__ out,
                                                 uint64_t n, const unsigned long long* gate) {
    if (gated_off(gate)) return;
    __shared__ unsigned long long s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (uint64_t base = 0; base < nb; base += SCAN_T) {
        const uint64_t i = base + threadIdx.x;
        const unsigned long long v = i < nb ? bsum[i] : 0;
        const unsigned long long incl = block_incl_sum_1024(v);
        const unsigned long long carry = s_carry;
        if (i < nb) bsum[i] = carry + incl - v;
        __syncthreads();
        if (threadIdx.x == SCAN_T - 1) s_carry = carry + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) out[n] = s_carry;
}
static __global__ __launch_bounds__(SCAN_T) void k_scanC(uint64_t* __restrict__ out, uint64_t n,
                                                 const uint64_t* __restrict__ bsum, const unsigned long long* gate) {
    if (gated_off(gate)) return;
    const uint64_t i0 = ((uint64_t)blockIdx.x * SCAN_T + threadIdx.x) * SCAN_PER;
    const uint64_t add = bsum[blockIdx.x];
#pragma unroll
    for (int q = 0; q < SCAN_PER; q++)
        if (i0 + q < n) out[i0 + q] += add;
}
static void launch_scan(const uint32_t* in, uint64_t n, uint64_t* out, uint64_t* bsum, hipStream_t s,
                        const unsigned long long* gate = nullptr) {
    const uint64_t per = (uint64_t)SCAN_T * SCAN_PER;
    const unsigned nb = (unsigned)((n + per - 1) / per);
    hipLaunchKernelGGL(k_scanA, dim3(nb), dim3(SCAN_T), 0, s, in, n, out, bsum, gate);
    hipLaunchKernelGGL(k_scanB, dim3(1), dim3(SCAN_T), 0, s, bsum, (uint64_t)nb, out, n, gate);
    hipLaunchKernelGGL(k_scanC, dim3(nb), dim3(SCAN_T), 0, s, out, n, bsum, gate);
}

// --------------------------------------------------------------------------------
// k_dump<W>: occupied slots with T(c) >= a -> records {W key words, T(c)}
// count_mode 0: c mod 65536 (-m 0); else min(c, 16383).  out == nullptr: count only.
// --------------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(256) void k_dump(TableView tv, int count_mode, uint64_t min_abundance,
                                              uint64_t* __restrict__ out, DevCounters* __restrict__ ctr) {
    constexpr int S = BUCKET_WORDS / (W + 1);
    const uint64_t bkt = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t occ = 0, nout = 0;
    uint64_t tv_c[S];
    bool emit[S];
    uint64_t bw[BUCKET_WORDS];
    if (bkt < tv.nbuckets) load_bucket(tv.buckets + bkt * BUCKET_WORDS, bw);
#pragma unroll
    for (int s = 0; s < S; s++) {
        emit[s] = false;
        tv_c[s] = 0;
        if (bkt < tv.nbuckets && bw[s * W] != EMPTY) {
            occ++;
            const uint64_t c = bw[S * W + s] & CNT_MASK;
            const uint64_t t = count_mode == 0 ? (c & 0xFFFF) : (c < 16383 ? c : 16383);
            if (t >= min_abundance) { emit[s] = true; tv_c[s] = t; nout++; }
        }
    }
    // output positions: one atomic per workgroup (not per wave) on the shared cursor
    __shared__ unsigned long long s_wt[4], s_base;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_sum(nout);
    if (lane == 63) s_wt[wid] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long tot = s_wt[0] + s_wt[1] + s_wt[2] + s_wt[3];
        s_base = tot ? atomicAdd(&ctr->dump_n, tot) : 0;
    }
    __syncthreads();
    unsigned long long base = s_base;
    for (int w = 0; w < wid; w++) base += s_wt[w];
    uint64_t idx = base + incl - nout;
#pragma unroll
    for (int s = 0; s < S; s++)
        if (out && emit[s]) {
            uint64_t t[W], key[W];
#pragma unroll
            for (int i = 0; i < W; i++) t[i] = bw[s * W + i];
            from_tkey<W>(t, key);
            uint64_t* o = out + idx * (W + 1);
#pragma unroll
            for (int i = 0; i < W; i++) o[i] = key[i];
            o[W] = tv_c[s];
            idx++;
        }
    block_add4(occ, 0, 0, 0, &ctr->occupied, nullptr, nullptr, nullptr);
}

// --------------------------------------------------------------------------------
// GPU output formatting: "<CANONICAL_KMER> <T(c)>\n" for every slot
// with T(c) >= a, in table order.  Replaces the reference's single-threaded writers
// write_kmers_on_disk_separately_even_faster (kmer_hash_table.cpp:4318-4524: chain walk,
// int2char, "<kmer> <count>\n") and write_kmers (2013-2050).  One workgroup formats
// TEXT_T consecutive buckets: k_text_bytes gives its byte count, the host scans them
// into block offsets, k_text writes the block's lines into LDS and copies them out
// contiguously at its offset (one text stream, no per-line atomics).
// --------------------------------------------------------------------------------
DEV uint32_t ndigits(uint32_t t) { return t >= 10000 ? 5 : t >= 1000 ? 4 : t >= 100 ? 3 : t >= 10 ? 2 : 1; }

// T(c) of each emitted slot (0 = no line: a >= 1 so an emitted T(c) is >= 1); returns
// the bucket's text bytes
template <int W, int S = BUCKET_WORDS / (W + 1)>
DEV uint32_t text_bucket(const TableView& tv, uint64_t bkt, int count_mode, uint64_t a, int k,
                         uint64_t (&bw)[BUCKET_WORDS], uint32_t (&tc)[S]) {
    uint32_t bytes = 0;
    if (bkt < tv.nbuckets) load_bucket(tv.buckets + bkt * BUCKET_WORDS, bw);
#pragma unroll
    for (int s = 0; s < S; s++) {
        tc[s] = 0;
        if (bkt < tv.nbuckets && bw[s * W] != EMPTY) {
            const uint64_t c = bw[S * W + s] & CNT_MASK;
            const uint64_t t = count_mode == 0 ? (c & 0xFFFF) : (c < 16383 ? c : 16383);
            if (t >= a) {
                tc[s] = (uint32_t)t;
                bytes += (uint32_t)k + 2 + ndigits((uint32_t)t);
            }
        }
    }
    return bytes;
}

template <int NT>
DEV uint32_t block_excl_sum(uint32_t v, uint32_t* s_w, uint32_t& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_sum(v);
    if (lane == 63) s_w[wid] = incl;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        const uint32_t x = s_w[w];
        base += w < wid ? x : 0;
        tot += x;
    }
    total = tot;
    return base + incl - v;
}

template <int W>
__global__ __launch_bounds__(TEXT_T) void k_text_bytes(TableView tv, int count_mode, uint64_t a, int k,
                                                       uint32_t* __restrict__ block_bytes) {
    constexpr int S = BUCKET_WORDS / (W + 1);
    __shared__ uint32_t s_w[TEXT_T / 64];
    uint64_t bw[BUCKET_WORDS];
    uint32_t tc[S];
    const uint32_t v = text_bucket<W>(tv, (uint64_t)blockIdx.x * TEXT_T + threadIdx.x, count_mode, a, k, bw, tc);
    uint32_t total;
    block_excl_sum<TEXT_T>(v, s_w, total);
    if (threadIdx.x == 0) block_bytes[blockIdx.x] = total;
}

// the lines of one bucket's emitted slots (tc[s] != 0) at p: "<KMER> <T(c)>\n" each, the
// k-mer's characters int2char'd from the canonical key (functions_strings.cpp:72-90)
template <int W, int S = BUCKET_WORDS / (W + 1)>
DEV void format_lines(const uint64_t (&bw)[BUCKET_WORDS], const uint32_t (&tc)[S], int k, uint8_t* p) {
    const int c0 = k - 32 * (W - 1);  // characters in key word 0 (the others hold 32)
#pragma unroll
    for (int s = 0; s < S; s++) {
        if (!tc[s]) continue;
        uint64_t t[W], key[W];
#pragma unroll
        for (int i = 0; i < W; i++) t[i] = bw[s * W + i];
        from_tkey<W>(t, key);
#pragma unroll
        for (int w = 0; w < W; w++) {
            const int nc = w == 0 ? c0 : 32;
            const uint64_t x = key[w];
            for (int q = nc - 1; q >= 0; q--) *p++ = (uint8_t)(0x54474341u >> (8 * ((x >> (2 * q)) & 3)));
        }
        *p++ = ' ';
        uint32_t cnt = tc[s];
        const uint32_t nd = ndigits(cnt);
        for (int d = (int)nd - 1; d >= 0; d--) {
            p[d] = (uint8_t)('0' + cnt % 10);
            cnt /= 10;
        }
        p[nd] = '\n';
        p += nd + 1;
    }
}

// --------------------------------------------------------------------------------
// Order-independent digest of the output text (kc_output_digest): the lines kc_write would
// write, each hashed with XXH64 (seed 0) over its bytes incl. '\n', summed mod 2^64 and XORed,
// plus the line count and the sum of T(c).  Equal for any line order, and additive over tables
// (the owners of a sharded job) and over partitions of the k-mer space (oracle/kc_digest.c), so a
// whole-job result is checked without sorting or moving its text.  One TEXT_T-bucket block per
// workgroup, its lines formatted into LDS as k_text does; out[4] = {lines, count sum, hash sum,
// hash xor}.
// --------------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(TEXT_T) void k_text_digest(TableView tv, int count_mode, uint64_t a, int k,
                                                        unsigned long long* __restrict__ out) {
    constexpr int S = BUCKET_WORDS / (W + 1);
    extern __shared__ uint8_t s_txt[];
    __shared__ uint32_t s_w[TEXT_T / 64];
    __shared__ unsigned long long s_red[4][TEXT_T / 64];
    uint64_t bw[BUCKET_WORDS];
    uint32_t tc[S];
    const uint32_t v = text_bucket<W>(tv, (uint64_t)blockIdx.x * TEXT_T + threadIdx.x, count_mode, a, k, bw, tc);
    uint32_t total;
    uint32_t pos = block_excl_sum<TEXT_T>(v, s_w, total);
    format_lines<W>(bw, tc, k, s_txt + pos);
    uint64_t lines = 0, csum = 0, hsum = 0, hxor = 0;
#pragma unroll
    for (int s = 0; s < S; s++) {
        if (!tc[s]) continue;
        const uint32_t len = (uint32_t)k + 2 + ndigits(tc[s]);
        const uint64_t h = xxh64_bytes(s_txt + pos, len, 0);
        lines++;
        csum += tc[s];
        hsum += h;
        hxor ^= h;
        pos += len;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        lines += __shfl_xor(lines, d, 64);
        csum += __shfl_xor(csum, d, 64);
        hsum += __shfl_xor(hsum, d, 64);
        hxor ^= __shfl_xor(hxor, d, 64);
    }
    const int wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_red[0][wid] = lines;
        s_red[1][wid] = csum;
        s_red[2][wid] = hsum;
        s_red[3][wid] = hxor;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < TEXT_T / 64; w++) {
            lines += s_red[0][w];
            csum += s_red[1][w];
            hsum += s_red[2][w];
            hxor ^= s_red[3][w];
        }
        if (lines) {
            atomicAdd(&out[0], (unsigned long long)lines);
            atomicAdd(&out[1], (unsigned long long)csum);
            atomicAdd(&out[2], (unsigned long long)hsum);
            atomicXor(&out[3], (unsigned long long)hxor);
        }
    }
}

// blocks [blk0, blk0 + grid) write at out + off[b] - base; dynamic LDS >= the largest
// block's bytes
template <int W>
__global__ __launch_bounds__(TEXT_T) void k_text(TableView tv, int count_mode, uint64_t a, int k, uint64_t blk0,
                                                 const uint64_t* __restrict__ off, uint64_t base,
                                                 uint8_t* __restrict__ out) {
    constexpr int S = BUCKET_WORDS / (W + 1);
    extern __shared__ uint8_t s_txt[];
    __shared__ uint32_t s_w[TEXT_T / 64];
    const uint64_t b = blk0 + blockIdx.x;
    uint64_t bw[BUCKET_WORDS];
    uint32_t tc[S];
    const uint32_t v = text_bucket<W>(tv, b * TEXT_T + threadIdx.x, count_mode, a, k, bw, tc);
    uint32_t total;
    const uint32_t pos = block_excl_sum<TEXT_T>(v, s_w, total);
    format_lines<W>(bw, tc, k, s_txt + pos);
    __syncthreads();
    uint8_t* o = out + (off[b] - base);
    // copy out: byte head up to a 4-byte boundary of the destination, then dwords
    const uint32_t head = (uint32_t)((4 - ((uintptr_t)o & 3)) & 3) < total ? (uint32_t)((4 - ((uintptr_t)o & 3)) & 3)
                                                                            : total;
    if (threadIdx.x < head) o[threadIdx.x] = s_txt[threadIdx.x];
    const uint32_t nw = (total - head) / 4;
    uint32_t* o4 = reinterpret_cast<uint32_t*>(o + head);
    for (uint32_t i = threadIdx.x; i < nw; i += TEXT_T) {
        const uint8_t* q = s_txt + head + 4 * i;
        o4[i] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
    }
    const uint32_t tail0 = head + 4 * nw;
    if (tail0 + threadIdx.x < total) o[tail0 + threadIdx.x] = s_txt[tail0 + threadIdx.x];
}

// ================================================================================
// launchers: templates over the key width W.  This file is compiled once per W
// (kc_count_w.hip with -DKC_W=1..8, the translation units build in parallel); the
// W-dispatch of the C ABI's launch_* entry points is kc_count.hip.
// ================================================================================
static uint64_t pow5_mod54(int e) {
    uint64_t r = 1;
    for (int i = 0; i < e; i++) r = (r * 5) & M54;
    return r;
}

template <int W>
static hipError_t launch_count_w(PackedView sym, uint64_t sym_bound, int k, int mode, TableView t, BloomView bf,
                                 DevCounters* ctr, hipStream_t s) {
    const unsigned grid = (unsigned)((sym_bound + tile_win<W>() - 1) / tile_win<W>());
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

template <class K>
static hipError_t set_smem(K kernel, size_t bytes) {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes);
}

static BinRegion coarse_bins(const TableView& t) { return BinRegion{t.R, t.f2bits, 0, 1}; }

template <int W, bool SEG, bool CNT = false, bool GATE = false>
static hipError_t launch_p3(TableView t, DevCounters* ctr, PartBufs pb, const unsigned long long* gate, int fresh,
                            hipStream_t s, BloomView bf = BloomView{}) {
    size_t sm3 = (size_t)BPR * BUCKET_WORDS * 8 + (size_t)BPR * 8;
    auto p3 = k_p3<W, SEG, CNT, GATE>;
    if constexpr (W == 1 && SEG && !CNT)
        if (pb.rec6) p3 = k_p3<1, true, false, GATE, true>;
    if (GATE) {
        // the filter-2 slice goes to LDS if two workgroups still fit a CU (80 KiB each) beside the
        // kernel's own static LDS (segment prefixes, block sums: its real size)
        hipFuncAttributes fa{};
        size_t stat = 2048;
        if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(p3)) == hipSuccess) stat = fa.sharedSizeBytes;
        const uint64_t maxb = bf.nblocks / t.R + 2;
        const size_t used = sm3 + stat;
        const size_t room = used < 80 * 1024 ? 80 * 1024 - used : 0;
        bf.slice_blocks = maxb * 32 <= room ? (uint32_t)maxb : 0;
        sm3 += (size_t)bf.slice_blocks * 32;
    }
    if (SEG && pb.B2 > MAX_SEG_GROUP) return hipErrorInvalidValue;
    hipError_t e = set_smem(p3, sm3);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(p3, dim3((unsigned)t.R), dim3(P3_THREADS), sm3, s, t, pb, ctr, gate, fresh, bf);
    return hipGetLastError();
}

// level 2 on the exact layout (after an exact level 1): items of IW words; `gate` as in k_p1
template <int IW>
static hipError_t part_level2_exact(TableView t, PartBufs pb, hipStream_t s, const unsigned long long* gate) {
    const size_t sm2 = part_smem<IW>(t.F2), sm2h = hist_smem(t.F2);
    hipError_t e;
    if ((e = set_smem(k_p2<IW, false>, sm2h)) != hipSuccess) return e;
    if ((e = set_smem(k_p2<IW, true>, sm2)) != hipSuccess) return e;
    hipLaunchKernelGGL((k_p2<IW, false>), dim3(t.F1 * pb.B2), dim3(COUNT_THREADS), sm2h, s, t, pb, gate);
    launch_scan(pb.hist2, t.R * pb.B2, pb.off2, pb.bsum, s, gate);
    hipLaunchKernelGGL((k_p2<IW, true>), dim3(t.F1 * pb.B2), dim3(COUNT_THREADS), sm2, s, t, pb, gate);
    return hipGetLastError();
}

// levels 2 and 3 on the exact layout (after an exact level 1); `gate` as in k_p1.
// CNT: the items are {W key words, count} records (W + 1 words each).  GATE: Bloom gate
// at level 3 (bf).
template <int W, bool CNT = false, bool GATE = false>
static hipError_t part_levels23(TableView t, DevCounters* ctr, PartBufs pb, hipStream_t s,
                                const unsigned long long* gate = nullptr, int fresh = 0, BloomView bf = BloomView{}) {
    hipError_t e = part_level2_exact<CNT ? W + 1 : W>(t, pb, s, gate);
    if (e != hipSuccess) return e;
    return launch_p3<W, false, CNT, GATE>(t, ctr, pb, gate, fresh, s, bf);
}

template <bool SEG>
static hipError_t launch_b3(BloomView bf, TableView ft, DevCounters* ctr, PartBufs pb, const unsigned long long* gate,
                            int fresh, hipStream_t s, int is = 1, int cntw = -1, int rec_phase = 0) {
    const uint32_t bpr = (uint32_t)(bf.nblocks / ft.R);
    // + wave queues (+ their count flags for records)
    const size_t sm = (size_t)bpr * BF_BLOCK_WORDS * 4 + (size_t)(B3_THREADS / 64) * 64 * (cntw >= 0 ? 12 : 8);
    if (SEG && pb.B2 > MAX_SEG_GROUP) return hipErrorInvalidValue;
    hipError_t e = set_smem(k_b3<SEG>, sm);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_b3<SEG>, dim3((unsigned)ft.R), dim3(B3_THREADS), sm, s, bf, bpr, pb, ctr, gate, fresh, is,
                       cntw, rec_phase);
    return hipGetLastError();
}

// level 1 from the symbol stream, exact layout: windows -> F bins by `bin`, keys into `out`
template <int W, int MODE, class Bin>
static hipError_t part_level1(PackedView sym, int k, BloomView bf, DevCounters* ctr, PartBufs pb, uint32_t F,
                              Bin bin, uint64_t* out, hipStream_t s, const unsigned long long* gate = nullptr) {
    const uint64_t pk = pow5_mod54(k), pkm1 = pow5_mod54(k - 1);
    const size_t sm1 = part_smem<p1_out_words(W, MODE)>(F), sm1h = hist_smem(F);
    hipError_t e;
    auto kh = k_p1<W, MODE, false, Bin, OutExact>;
    auto ks = k_p1<W, MODE, true, Bin, OutExact>;
    if ((e = set_smem(kh, sm1h)) != hipSuccess) return e;
    if ((e = set_smem(ks, sm1)) != hipSuccess) return e;
    // a gated launch is the fallback of a segmented batch, whose windows are counted
    const int count = gate ? 0 : 1;
    hipLaunchKernelGGL(kh, dim3(pb.nblk1), dim3(COUNT_THREADS), sm1h, s, sym, k, bf, ctr, pb, F, bin, out, pk, pkm1,
                       OutExact{}, gate, count);
    launch_scan(pb.hist1, (uint64_t)F * pb.nblk1, pb.off1, pb.bsum, s, gate);
    hipLaunchKernelGGL(ks, dim3(pb.nblk1), dim3(COUNT_THREADS), sm1, s, sym, k, bf, ctr, pb, F, bin, out, pk, pkm1,
                       OutExact{}, gate, 0);
    return hipGetLastError();
}

// The skew list of a segmented batch, after its level 3 (its length is on the device):
// {key words, count} records -- keys that overflowed a segment (count 1) and the heavy
// records of repeated windows -- through the exact pipeline (levels 1-3 by histogram
// offsets, no capacity limits), behind the Bloom gate in the gated pass.  (The Bloom pass
// spills plain table-key words: bloom_part_w.)
template <int W, bool GATE>
static hipError_t insert_spill(TableView t, BloomView bf, DevCounters* ctr, PartBufs pb, hipStream_t s) {
    constexpr int IW = W + 1;
    const BinRegion bin = coarse_bins(t);
    const size_t sm1 = part_smem<IW>(t.F1), sm1h = hist_smem(t.F1);
    hipError_t e;
    if ((e = set_smem(k_p1k<IW, false>, sm1h)) != hipSuccess) return e;
    if ((e = set_smem(k_p1k<IW, true>, sm1)) != hipSuccess) return e;
    const DevN dn{&ctr->spill_n, pb.spill_cap, &ctr->part_overflow};
    hipLaunchKernelGGL((k_p1k<IW, false>), dim3(pb.nblk1), dim3(COUNT_THREADS), sm1h, s, pb.spill, (uint64_t)0, pb,
                       t.F1, bin, ctr, W, dn, IW);
    launch_scan(pb.hist1, (uint64_t)t.F1 * pb.nblk1, pb.off1, pb.bsum, s);
    hipLaunchKernelGGL((k_p1k<IW, true>), dim3(pb.nblk1), dim3(COUNT_THREADS), sm1, s, pb.spill, (uint64_t)0, pb,
                       t.F1, bin, ctr, W, dn, IW);
    return part_levels23<W, true, GATE>(t, ctr, pb, s, nullptr, 0, bf);
}

// Segmented level 2 of the table's geometry t: the default workgroup, or half of it when the
// F2 bins' arrays do not fit beside the full tile (wide keys in big tables, e.g. C5: k = 127,
// a 1.25 G-slot share; kc_api.cpp alloc_table picks F2 for it)
template <int W>
static hipError_t launch_p2f(TableView t, PartBufs pb, DevCounters* ctr, int rec, hipStream_t s, uint32_t pad = 0) {
    constexpr int NT = p2f_threads<W>(), NH = NT / 2;
    const uint32_t nseg = std::max<uint32_t>(pad, (pb.nblk1 + pb.B2 - 1) / pb.B2);
    hipError_t e;
    const size_t sm = p2f_smem<W, NT>(t.F2, nseg);
    if constexpr (W == 1) {
        if (pb.rec6) {  // 6-byte level-2 records, + the F2 regions' xlo in LDS
            if ((e = set_smem(k_p2f<1, NT, 1, true>, sm + (size_t)t.F2 * 4)) != hipSuccess) return e;
            hipLaunchKernelGGL((k_p2f<1, NT, 1, true>), dim3(t.F1 * pb.B2), dim3(NT), sm + (size_t)t.F2 * 4, s, t, pb,
                               ctr, rec);
            return hipGetLastError();
        }
    }
    if (sm <= LDS_BYTES || W <= 2) {
        if ((e = set_smem(k_p2f<W, NT>, sm)) != hipSuccess) return e;
        hipLaunchKernelGGL((k_p2f<W, NT>), dim3(t.F1 * pb.B2), dim3(NT), sm, s, t, pb, ctr, rec);
    } else {
        const size_t smh = p2f_smem<W, NH>(t.F2, nseg);
        if ((e = set_smem(k_p2f<W, NH>, smh)) != hipSuccess) return e;
        hipLaunchKernelGGL((k_p2f<W, NH>), dim3(t.F1 * pb.B2), dim3(NH), smh, s, t, pb, ctr, rec);
    }
    return hipGetLastError();
}

// batch bookkeeping of the skew lists: begin = clear the batch's flag and list counts,
// end = add the lists' lengths to the job totals
static __global__ void k_batch_begin(DevCounters* ctr) {
    ctr->part_overflow = 0;
    ctr->spill_n = 0;
    ctr->heavy_n = 0;
}
static __global__ void k_batch_end(DevCounters* ctr) {
    if (ctr->part_overflow) return;
    ctr->spilled += ctr->spill_n - ctr->heavy_n;  // list entries: spilled keys + heavy records
    ctr->heavy += ctr->heavy_n;
}

// Rec12 in the table's geometry (R12_REG): a coarse bin spans at most ceil(F2 * 2^32 / R) values
// of x, a region ceil(2^32 / R); level 1 (k_p1 -> k_p2f) and level 2 (k_p2f -> k_p3) take the
// 12-byte records independently, each when hb + 1 + xb <= 32 (else 16-byte records)
static inline void set_rec12_table(PartBufs& pb, const TableView& t, int k) {
    pb.rec12 = 0;
    if (t.R == 0) return;
    const int hb = std::max(0, 2 * k - 96);
    const uint64_t f2 = 1ULL << t.f2bits;
    const int xb1 = span_bits32(((f2 << 32) + t.R - 1) / t.R), xb2 = span_bits32(((1ULL << 32) + t.R - 1) / t.R);
    if (hb + 1 + xb1 <= 32) {
        pb.rec12 |= R12_P1 | R12_IN;
        pb.r12_xb1 = xb1;
    }
    if (hb + 1 + xb2 <= 32) {
        pb.rec12 |= R12_OUT | R12_L2;
        pb.r12_xb2 = xb2;
    }
    if (pb.rec12) pb.rec12 |= R12_REG;
    pb.r12_hb = hb;
    pb.r12_b2s = 0;
}

// Segmented pipeline (pb.cap1 != 0): p1 -> p2f -> p3<SEG>, each a single pass; then
// the exact pipeline behind the overflow gate (its kernels return at once unless a
// segment overflowed, in which case the segmented p3 left the table untouched).
template <int W, int MODE>
static hipError_t launch_part_w(PackedView sym, int k, TableView t, BloomView bf, DevCounters* ctr, PartBufs pb,
                                int fresh, hipStream_t s, int phase) {
    constexpr bool GATE3 = MODE == 4;
    if (pb.cap1 == 0) {
        if (!(phase & PH_MAIN)) return hipSuccess;
        hipError_t e = part_level1<W, MODE>(sym, k, bf, ctr, pb, t.F1, coarse_bins(t), pb.keys1, s);
        if (e != hipSuccess) return e;
        return part_levels23<W, false, GATE3>(t, ctr, pb, s, nullptr, fresh, bf);
    }
    hipError_t e;
    const unsigned long long* gate = &ctr->part_overflow;
    // one-word keys in a table of >= 2^16 regions: 6-byte level-2 records (StoreRec6)
    pb.rec6 = W == 1 && t.R >= (1ULL << 16);
    // two-word keys: 12-byte records at each level whose bins span few enough values of x
    if constexpr (W == 2) set_rec12_table(pb, t, k);
    if (phase & PH_L3) {  // the deferred level 3 of a group of batches: B2 = the group's segments
        PartBufs p3 = pb;
        p3.B2 = pb.b2t;
        p3.b2t = p3.b2off = 0;
        if ((e = launch_p3<W, true, false, GATE3>(t, ctr, p3, nullptr, fresh, s, bf)) != hipSuccess) return e;
    }
    if (phase & (PH_MAIN | PH_L12)) {
    if (!pb.keep_skew) hipLaunchKernelGGL(k_batch_begin, dim3(1), dim3(1), 0, s, ctr);
    const uint64_t pk = pow5_mod54(k), pkm1 = pow5_mod54(k - 1);
    auto k1 = k_p1<W, MODE, true, BinRegion, OutSeg, scatter_threads<W>()>;
    // Short level-1 runs (fewer than 8 keys per bin and tile: big tables, C4 shares) leave
    // partial 128-byte lines that L2 merges only while they stay resident: one workgroup per
    // CU halves the open lines (C4 share: k_p1 writes 33 GB for 20 GB of keys; count
    // 41.0 -> 40.15 ms; C2's 34-key runs lose 18 % that way, profiles/r02_v16_ab_p1_lds.txt)
    const size_t p1_lds_min = (size_t)p1_tile(W) < 8 * (size_t)t.F1 ? LDS_BYTES / 2 + 16 : 0;
    const size_t sm1 = std::max(p1_lds_min, p1_smem<W, W, scatter_threads<W>()>(t.F1) + heavy_smem<W>() +
                                                p1_stage_smem<W, scatter_threads<W>()>());
    const OutSeg o1{(uint64_t)pb.nblk1 * pb.cap1, 0, pb.cap1, pb.spill, pb.spill_cap, &ctr->spill_n,
                    &ctr->part_overflow, 1};
    bool wide = false;
    if constexpr (W == 2) {  // (kc_internal.h p1_wide: big tables' two-word level 1)
        if (p1_wide(W, t.F1)) {
            wide = true;
            auto kw = k_p1<W, MODE, true, BinRegion, OutSeg, P1_WIDE_THREADS>;
            const size_t smw = p1_smem<W, W, P1_WIDE_THREADS>(t.F1) + heavy_smem<W>() + p1_stage_smem<W, P1_WIDE_THREADS>();
            if ((e = set_smem(kw, smw)) != hipSuccess) return e;
            hipLaunchKernelGGL(kw, dim3(pb.nblk1), dim3(P1_WIDE_THREADS), smw, s, sym, k, bf, ctr, pb, t.F1,
                               coarse_bins(t), pb.keys1, pk, pkm1, o1, (const unsigned long long*)nullptr, 1);
        }
    }
    if (!wide) {
        if ((e = set_smem(k1, sm1)) != hipSuccess) return e;
        hipLaunchKernelGGL(k1, dim3(pb.nblk1), dim3(scatter_threads<W>()), sm1, s, sym, k, bf, ctr, pb, t.F1,
                           coarse_bins(t), pb.keys1, pk, pkm1, o1, (const unsigned long long*)nullptr, 1);
    }
    if ((e = launch_p2f<W>(t, pb, ctr, 1, s)) != hipSuccess) return e;
    if (phase & PH_MAIN)
        if ((e = launch_p3<W, true, false, GATE3>(t, ctr, pb, nullptr, fresh, s, bf)) != hipSuccess) return e;
    }
    if (!(phase & PH_TAIL)) return hipGetLastError();
    // the skew lists (MODE 2 rolls its windows: no heavy records); the segmented level 3
    // wrote every region of a fresh table, so these read the table
    if ((e = insert_spill<W, GATE3>(t, bf, ctr, pb, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_batch_end, dim3(1), dim3(1), 0, s, ctr);
    // a full spill or heavy list: the exact pipeline redoes the batch (the segmented levels
    // and the lists left the table untouched)
    if ((e = part_level1<W, MODE>(sym, k, bf, ctr, pb, t.F1, coarse_bins(t), pb.keys1, s, gate)) != hipSuccess)
        return e;
    return part_levels23<W, false, GATE3>(t, ctr, pb, s, gate, fresh, bf);
}

// mode 2 (counting behind the Bloom gate): blocked layout -> gate at level 3 (MODE 4),
// reference layout -> gate on the rolled root at level 1 (MODE 2)
template <int W>
static hipError_t count_part_w(PackedView sym, int k, int mode, TableView t, BloomView bf, DevCounters* ctr,
                               PartBufs pb, int fresh, hipStream_t s, int phase) {
    if (mode != 2) return launch_part_w<W, 0>(sym, k, t, bf, ctr, pb, fresh, s, phase);
    if (bf.blocked) return launch_part_w<W, 4>(sym, k, t, bf, ctr, pb, fresh, s, phase);
    return launch_part_w<W, 2>(sym, k, t, bf, ctr, pb, fresh, s, phase);
}
// Bloom pass 1 on the blocked layout, partitioned: windows -> table key word 0 -> coarse
// bins -> filter regions (ft: R = filter regions, F1 x F2) -> k_b3 (LDS-resident filter
// regions).  Segmented single passes with the exact pipeline behind the overflow gate,
// as for the table.
// KEEP (partition reuse, kc_api.cpp): levels 1 and 2 move the whole table key (MODE 5) and
// partition by fg, a power-of-two geometry at least as fine as the filter regions ft; k_b3
// reads word 0 of each filter region's fine bins (consecutive, B2 x R_fine / R_f segments).
// A table of the same hash-prefix bins can then be counted from these partitions: from level
// 2 (its regions are unions of fine bins) or from level 1 (its coarse bins are fg's).  The
// segment fills of both levels are copied aside (the skew-list pass reuses hist1 / hist2).
template <int W, bool KEEP>
static hipError_t bloom_part_w(PackedView sym, int k, BloomView bf, TableView ft, TableView fg, DevCounters* ctr,
                               PartBufs pb, int fresh, hipStream_t s, int phase) {
    if (pb.cap1 == 0) {
        if (!(phase & PH_MAIN)) return hipSuccess;
        hipError_t e = part_level1<W, 3>(sym, k, bf, ctr, pb, ft.F1, coarse_bins(ft), pb.keys1, s);
        if (e != hipSuccess) return e;
        if ((e = part_level2_exact<1>(ft, pb, s, nullptr)) != hipSuccess) return e;
        return launch_b3<false>(bf, ft, ctr, pb, nullptr, fresh, s);
    }
    constexpr int MODE = KEEP ? 5 : 3, OW = KEEP ? W : 1;
    const TableView& lg = KEEP ? fg : ft;  // the partition levels' geometry
    hipError_t e;
    const unsigned long long* gate = &ctr->part_overflow;
    if (phase & PH_MAIN) {
    hipLaunchKernelGGL(k_batch_begin, dim3(1), dim3(1), 0, s, ctr);
    const uint64_t pk = pow5_mod54(k), pkm1 = pow5_mod54(k - 1);
    constexpr int NT = scatter_threads<W>(), NT2 = p2f_threads<OW>();
    auto k1 = k_p1<W, MODE, true, BinRegion, OutSeg, NT>;
    auto k2 = k_p2f<OW, NT2>;
    const size_t sm1 = p1_smem<W, OW, NT>(lg.F1) + heavy_smem<OW>() + p1_stage_smem<W, NT>(),
                 sm2 = p2f_smem<OW, NT2>(lg.F2, (pb.nblk1 + pb.B2 - 1) / pb.B2);
    if ((e = set_smem(k1, sm1)) != hipSuccess) return e;
    if ((e = set_smem(k2, sm2)) != hipSuccess) return e;
    const OutSeg o1{(uint64_t)pb.nblk1 * pb.cap1, 0, pb.cap1, pb.spill, pb.spill_cap, &ctr->spill_n,
                    &ctr->part_overflow, 0};
    hipLaunchKernelGGL(k1, dim3(pb.nblk1), dim3(NT), sm1, s, sym, k, bf, ctr, pb, lg.F1, coarse_bins(lg), pb.keys1, pk,
                       pkm1, o1, (const unsigned long long*)nullptr, 1);
    hipLaunchKernelGGL(k2, dim3(lg.F1 * pb.B2), dim3(NT2), sm2, s, lg, pb, ctr, 0);
    if constexpr (KEEP) {
        if (pb.keep_fill &&
            ((e = hipMemcpyAsync(pb.keep_fill, pb.hist1, (size_t)fg.F1 * pb.nblk1 * 4, hipMemcpyDeviceToDevice, s)) !=
                 hipSuccess ||
             (e = hipMemcpyAsync(pb.keep_fill2, pb.hist2, (size_t)fg.R * pb.B2 * 4, hipMemcpyDeviceToDevice, s)) !=
                 hipSuccess))
            return e;
    }
    }
    if (phase & PH_MAIN) {
        PartBufs p3 = pb;  // k_b3's view: a filter region = R_fine / R_f consecutive fine bins
        if constexpr (KEEP) p3.B2 = (uint32_t)(fg.R / ft.R) * pb.B2;
        if ((e = launch_b3<true>(bf, ft, ctr, p3, nullptr, fresh, s, OW)) != hipSuccess) return e;
    }
    if (!(phase & PH_TAIL)) return hipGetLastError();
    // spilled keys (table key word 0 of OW-word entries) through the exact levels into the
    // filter regions
    {
        const BinRegion bin = coarse_bins(ft);
        const size_t s1 = part_smem<1>(ft.F1), s1h = hist_smem(ft.F1);
        if ((e = set_smem(k_p1k<1, false>, s1h)) != hipSuccess) return e;
        if ((e = set_smem(k_p1k<1, true>, s1)) != hipSuccess) return e;
        const DevN dn{&ctr->spill_n, pb.spill_cap, &ctr->part_overflow};
        hipLaunchKernelGGL((k_p1k<1, false>), dim3(pb.nblk1), dim3(COUNT_THREADS), s1h, s, pb.spill, (uint64_t)0, pb,
                           ft.F1, bin, ctr, -1, dn, OW);
        launch_scan(pb.hist1, (uint64_t)ft.F1 * pb.nblk1, pb.off1, pb.bsum, s);
        hipLaunchKernelGGL((k_p1k<1, true>), dim3(pb.nblk1), dim3(COUNT_THREADS), s1, s, pb.spill, (uint64_t)0, pb,
                           ft.F1, bin, ctr, -1, dn, OW);
        if ((e = part_level2_exact<1>(ft, pb, s, nullptr)) != hipSuccess) return e;
        if ((e = launch_b3<false>(bf, ft, ctr, pb, nullptr, 0, s)) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_batch_end, dim3(1), dim3(1), 0, s, ctr);
    if ((e = part_level1<W, 3>(sym, k, bf, ctr, pb, ft.F1, coarse_bins(ft), pb.keys1, s, gate)) != hipSuccess)
        return e;
    if ((e = part_level2_exact<1>(ft, pb, s, gate)) != hipSuccess) return e;
    return launch_b3<false>(bf, ft, ctr, pb, gate, fresh, s);
}

// The counting pass of a job whose Bloom pass kept its partitions (bloom_part_w KEEP):
// level >= 2: pb.keys2 / hist2 / cap2 are the fine bins and pb.B2 the fine bins per table
// region times their segments (the regions are unions of fine bins): level 3 only; level 1:
// pb.keys1 / hist1 / cap1 / nblk1 / B2 are the kept level 1 (the table's coarse bins are
// the fine geometry's): levels 2 and 3.  Then the skew list and the batch's windows (counted
// by the Bloom pass).
static __global__ void k_add_windows(DevCounters* ctr, unsigned long long n) {
    if (!ctr->part_overflow) ctr->windows += n;
}
static __global__ void k_add_inserted(DevCounters* ctr, unsigned long long n) {
    if (!ctr->part_overflow) ctr->inserted += n;
}
template <int W, bool GATE>
static hipError_t count_reuse_w(TableView t, BloomView bf, DevCounters* ctr, PartBufs pb, int fresh, int level,
                                uint64_t windows, hipStream_t s) {
    hipError_t e;
    hipLaunchKernelGGL(k_batch_begin, dim3(1), dim3(1), 0, s, ctr);
    if (level < 2) {
        if ((e = launch_p2f<W>(t, pb, ctr, 1, s)) != hipSuccess) return e;
    }
    if ((e = launch_p3<W, true, false, GATE>(t, ctr, pb, nullptr, fresh, s, bf)) != hipSuccess) return e;
    // (from level 2 nothing can reach the skew list: no level of this pass scatters)
    if (level < 2 && (e = insert_spill<W, GATE>(t, bf, ctr, pb, s)) != hipSuccess) return e;
    // ungated (-m 1 -b): every window is an insertion (level 1 counts them in an ordinary pass)
    if (!GATE) hipLaunchKernelGGL(k_add_inserted, dim3(1), dim3(1), 0, s, ctr, (unsigned long long)windows);
    hipLaunchKernelGGL(k_batch_end, dim3(1), dim3(1), 0, s, ctr);
    hipLaunchKernelGGL(k_add_windows, dim3(1), dim3(1), 0, s, ctr, (unsigned long long)windows);
    return hipGetLastError();
}

// Routing for hash-prefix sharding: windows -> table keys grouped by owner shard into
// `out`; per-owner offsets in pb.off1 ([owner][block], exclusive, last entry = total).
template <int W>
static hipError_t route_w(PackedView sym, int k, DevCounters* ctr, PartBufs pb, uint32_t parts, uint64_t* out,
                          hipStream_t s) {
    return part_level1<W, 0>(sym, k, BloomView{}, ctr, pb, parts, BinOwner{parts}, out, s);
}
// Insert an array of table keys (e.g. received from other shards), or, CNT, of
// {W key words, count} records (shard merge), partitioned through the exact pipeline.
template <int W, bool CNT>
static hipError_t insert_items_part(const uint64_t* items, uint64_t n, TableView t, DevCounters* ctr, PartBufs pb,
                                    int fresh, hipStream_t s) {
    constexpr int IW = CNT ? W + 1 : W;
    const BinRegion bin = coarse_bins(t);
    const size_t sm1 = part_smem<IW>(t.F1), sm1h = hist_smem(t.F1);
    hipError_t e;
    if ((e = set_smem(k_p1k<IW, false>, sm1h)) != hipSuccess) return e;
    if ((e = set_smem(k_p1k<IW, true>, sm1)) != hipSuccess) return e;
    const int cw = CNT ? W : -1;
    hipLaunchKernelGGL((k_p1k<IW, false>), dim3(pb.nblk1), dim3(COUNT_THREADS), sm1h, s, items, n, pb, t.F1, bin, ctr,
                       cw, DevN{}, IW);
    launch_scan(pb.hist1, (uint64_t)t.F1 * pb.nblk1, pb.off1, pb.bsum, s);
    hipLaunchKernelGGL((k_p1k<IW, true>), dim3(pb.nblk1), dim3(COUNT_THREADS), sm1, s, items, n, pb, t.F1, bin, ctr,
                       cw, DevN{}, IW);
    return part_levels23<W, CNT>(t, ctr, pb, s, nullptr, fresh);
}


// Bloom pass 1 over pre-aggregated {key, count} records of distinct keys (kc_bloom_records_device,
// the owner side of the sharded Bloom filter): the exact levels move whole records into the
// filter's regions (ft); k_b3 inserts the records of count >= 2 twice, then (a second launch) the
// others once
template <int W>
static hipError_t bloom_records_w(const uint64_t* rec, uint64_t n, BloomView bf, TableView ft, DevCounters* ctr,
                                  PartBufs pb, int fresh, hipStream_t s) {
    constexpr int IW = W + 1;
    if (n == 0) return hipSuccess;
    const BinRegion bin = coarse_bins(ft);
    const size_t sm1 = part_smem<IW>(ft.F1), sm1h = hist_smem(ft.F1);
    hipError_t e;
    if ((e = set_smem(k_p1k<IW, false>, sm1h)) != hipSuccess) return e;
    if ((e = set_smem(k_p1k<IW, true>, sm1)) != hipSuccess) return e;
    hipLaunchKernelGGL((k_p1k<IW, false>), dim3(pb.nblk1), dim3(COUNT_THREADS), sm1h, s, rec, n, pb, ft.F1, bin, ctr, -2,
                       DevN{}, IW);
    launch_scan(pb.hist1, (uint64_t)ft.F1 * pb.nblk1, pb.off1, pb.bsum, s);
    hipLaunchKernelGGL((k_p1k<IW, true>), dim3(pb.nblk1), dim3(COUNT_THREADS), sm1, s, rec, n, pb, ft.F1, bin, ctr, -2,
                       DevN{}, IW);
    if ((e = part_level2_exact<IW>(ft, pb, s, nullptr)) != hipSuccess) return e;
    // the k-mers seen at least twice first (filters 1 and 2), then the singletons
    if ((e = launch_b3<false>(bf, ft, ctr, pb, nullptr, fresh, s, IW, W, 0)) != hipSuccess) return e;
    return launch_b3<false>(bf, ft, ctr, pb, nullptr, 0, s, IW, W, 1);
}

// the counting pass over {key, count} records behind the gate (kc_count_records_device): the
// exact levels into the table's regions, k_p3<CNT, GATE> adds the counts of the records whose
// filter-2 bits are set (inserted += those counts); gate = 0: every record
template <int W>
static hipError_t count_records_w(const uint64_t* rec, uint64_t n, TableView t, BloomView bf, DevCounters* ctr,
                                  PartBufs pb, int fresh, int gate, hipStream_t s) {
    constexpr int IW = W + 1;
    if (n == 0) return hipSuccess;
    const BinRegion bin = coarse_bins(t);
    const size_t sm1 = part_smem<IW>(t.F1), sm1h = hist_smem(t.F1);
    hipError_t e;
    if ((e = set_smem(k_p1k<IW, false>, sm1h)) != hipSuccess) return e;
    if ((e = set_smem(k_p1k<IW, true>, sm1)) != hipSuccess) return e;
    const int cw = gate ? -2 : W;  // gated: level 3 counts what passes
    hipLaunchKernelGGL((k_p1k<IW, false>), dim3(pb.nblk1), dim3(COUNT_THREADS), sm1h, s, rec, n, pb, t.F1, bin, ctr, cw,
                       DevN{}, IW);
    launch_scan(pb.hist1, (uint64_t)t.F1 * pb.nblk1, pb.off1, pb.bsum, s);
    hipLaunchKernelGGL((k_p1k<IW, true>), dim3(pb.nblk1), dim3(COUNT_THREADS), sm1, s, rec, n, pb, t.F1, bin, ctr, cw,
                       DevN{}, IW);
    if (gate) return part_levels23<W, true, true>(t, ctr, pb, s, nullptr, fresh, bf);
    return part_levels23<W, true>(t, ctr, pb, s, nullptr, fresh);
}

template <int W>
static hipError_t insert_keys_w(const uint64_t* keys, uint64_t n, bool partitioned, TableView t, DevCounters* ctr,
                                PartBufs pb, int fresh, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (!partitioned) {
        hipLaunchKernelGGL((k_insert_keys<W>), dim3((unsigned)((n + COUNT_THREADS - 1) / COUNT_THREADS)),
                           dim3(COUNT_THREADS), 0, s, keys, n, t, ctr);
        return hipGetLastError();
    }
    return insert_items_part<W, false>(keys, n, t, ctr, pb, fresh, s);
}
template <int W>
static hipError_t text_w(TableView t, int count_mode, uint64_t a, int k, uint64_t blk0, uint64_t nblk,
                         const uint64_t* off, uint64_t base, uint8_t* out, size_t lds, hipStream_t s) {
    auto kern = k_text<W>;
    hipError_t e = set_smem(kern, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(TEXT_T), lds, s, t, count_mode, a, k, blk0, off, base, out);
    return hipGetLastError();
}

template <int W>
static hipError_t insert_runs_w(const uint64_t* rec, const uint64_t* gstart, uint32_t G, TableView t,
                                DevCounters* ctr, uint32_t* m_len, uint64_t* m_start, int fresh, hipStream_t s) {
    const uint64_t nb = (t.R + 1) * G;
    hipLaunchKernelGGL(k_run_bounds<W>, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, rec, gstart, G, t.R,
                       m_start);
    hipLaunchKernelGGL(k_run_lengths, dim3((unsigned)((t.R * G + 255) / 256)), dim3(256), 0, s, m_start, t.R * G, G,
                       m_len);
    PartBufs pb{};
    pb.B2 = G;
    pb.hist2 = m_len;
    pb.keys2 = const_cast<uint64_t*>(rec);
    pb.seg_start = m_start;
    return launch_p3<W, true, true>(t, ctr, pb, nullptr, fresh, s);
}
// ---- the W-specific entry points (declared in kc_internal.h, dispatched by kc_count.hip) ----
template <int W>
hipError_t WOps<W>::count(PackedView sym, uint64_t sym_bound, int k, int mode, TableView t, BloomView bf,
                          DevCounters* ctr, hipStream_t s) {
    return launch_count_w<W>(sym, sym_bound, k, mode, t, bf, ctr, s);
}

template <int W>
hipError_t WOps<W>::count_partitioned(PackedView sym, int k, int mode, TableView t, BloomView bf, DevCounters* ctr,
                                      PartBufs pb, int fresh, hipStream_t s, int phase) {
    return count_part_w<W>(sym, k, mode, t, bf, ctr, pb, fresh, s, phase);
}

template <int W>
hipError_t WOps<W>::bloom_partitioned(PackedView sym, int k, BloomView bf, TableView ft, TableView fg, DevCounters* ctr,
                                      PartBufs pb, int fresh, int keep, hipStream_t s, int phase) {
    if (keep) return bloom_part_w<W, true>(sym, k, bf, ft, fg, ctr, pb, fresh, s, phase);
    return bloom_part_w<W, false>(sym, k, bf, ft, fg, ctr, pb, fresh, s, phase);
}
template <int W>
hipError_t WOps<W>::count_reuse(TableView t, BloomView bf, DevCounters* ctr, PartBufs pb, int fresh, int level,
                                int gate, uint64_t windows, hipStream_t s) {
    if (gate) return count_reuse_w<W, true>(t, bf, ctr, pb, fresh, level, windows, s);
    return count_reuse_w<W, false>(t, bf, ctr, pb, fresh, level, windows, s);
}

template <int W>
hipError_t WOps<W>::bloom_records(const uint64_t* rec, uint64_t n, BloomView bf, TableView ft, DevCounters* ctr,
                                  PartBufs pb, int fresh, hipStream_t s) {
    return bloom_records_w<W>(rec, n, bf, ft, ctr, pb, fresh, s);
}
template <int W>
hipError_t WOps<W>::count_records(const uint64_t* rec, uint64_t n, TableView t, BloomView bf, DevCounters* ctr,
                                  PartBufs pb, int fresh, int gate, hipStream_t s) {
    return count_records_w<W>(rec, n, t, bf, ctr, pb, fresh, gate, s);
}

template <int W>
hipError_t WOps<W>::route(PackedView sym, int k, DevCounters* ctr, PartBufs pb, uint32_t parts, uint64_t* out,
                          hipStream_t s) {
    return route_w<W>(sym, k, ctr, pb, parts, out, s);
}

template <int W>
hipError_t WOps<W>::insert_keys(const uint64_t* keys, uint64_t n, bool partitioned, TableView t, DevCounters* ctr,
                                PartBufs pb, int fresh, hipStream_t s) {
    return insert_keys_w<W>(keys, n, partitioned, t, ctr, pb, fresh, s);
}

template <int W>
hipError_t WOps<W>::route_table(TableView t, uint32_t parts, uint32_t* hist, uint64_t* off, uint64_t* bsum,
                                uint64_t* out, hipStream_t s, int hist_ready) {
    const unsigned nblk = (unsigned)((t.nbuckets + 255) / 256);
    if (!out) {
        if (!hist_ready)
            hipLaunchKernelGGL((k_route_table<W, false>), dim3(nblk), dim3(256), 0, s, t, parts, hist, off, out);
        launch_scan(hist, (uint64_t)parts * nblk, off, bsum, s);
    } else {
        hipLaunchKernelGGL((k_route_table<W, true>), dim3(nblk), dim3(256), 0, s, t, parts, hist, off, out);
    }
    return hipGetLastError();
}

template <int W>
hipError_t WOps<W>::insert_counts(const uint64_t* rec, uint64_t n, bool partitioned, TableView t, DevCounters* ctr,
                                  PartBufs pb, int fresh, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (partitioned) return insert_items_part<W, true>(rec, n, t, ctr, pb, fresh, s);
    const dim3 grid((unsigned)((n + COUNT_THREADS - 1) / COUNT_THREADS));
    hipLaunchKernelGGL(k_insert_counts<W>, grid, dim3(COUNT_THREADS), 0, s, rec, n, t, ctr);
    return hipGetLastError();
}

template <int W>
hipError_t WOps<W>::check_runs(const uint64_t* rec, const uint64_t* gstart, uint32_t G, uint64_t maxn, TableView t,
                               unsigned long long* flag, hipStream_t s) {
    const dim3 grid((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(1024, (maxn + 255) / 256)), G);
    hipLaunchKernelGGL(k_check_runs<W>, grid, dim3(256), 0, s, rec, gstart, t.R, flag);
    return hipGetLastError();
}

template <int W>
hipError_t WOps<W>::insert_counts_runs(const uint64_t* rec, const uint64_t* gstart, uint32_t G, TableView t,
                                       DevCounters* ctr, uint32_t* m_len, uint64_t* m_start, int fresh, hipStream_t s) {
    return insert_runs_w<W>(rec, gstart, G, t, ctr, m_len, m_start, fresh, s);
}

template <int W>
hipError_t WOps<W>::dump(TableView t, int count_mode, uint64_t min_abundance, uint64_t* out, DevCounters* ctr,
                         hipStream_t s) {
    const unsigned grid = (unsigned)((t.nbuckets + 255) / 256);
    hipLaunchKernelGGL(k_dump<W>, dim3(grid), dim3(256), 0, s, t, count_mode, min_abundance, out, ctr);
    return hipGetLastError();
}

template <int W>
hipError_t WOps<W>::text_bytes(TableView t, int count_mode, uint64_t a, int k, uint32_t* block_bytes, uint64_t* off,
                               uint64_t* bsum, hipStream_t s) {
    const uint64_t nblk = (t.nbuckets + TEXT_T - 1) / TEXT_T;
    hipLaunchKernelGGL(k_text_bytes<W>, dim3((unsigned)nblk), dim3(TEXT_T), 0, s, t, count_mode, a, k, block_bytes);
    launch_scan(block_bytes, nblk, off, bsum, s);
    return hipGetLastError();
}

template <int W>
hipError_t WOps<W>::text(TableView t, int count_mode, uint64_t a, int k, uint64_t blk0, uint64_t nblk,
                         const uint64_t* off, uint64_t base, uint8_t* out, size_t lds, hipStream_t s) {
    return text_w<W>(t, count_mode, a, k, blk0, nblk, off, base, out, lds, s);
}

template <int W>
hipError_t WOps<W>::text_digest(TableView t, int count_mode, uint64_t a, int k, unsigned long long* out,
                                hipStream_t s) {
    // every block's lines fit: TEXT_T buckets x S slots x (k + 2 + 5) bytes (<= 124 KiB for k <= 479)
    const size_t lds = ((size_t)TEXT_T * (BUCKET_WORDS / (W + 1)) * ((size_t)k + 7) + 15) / 16 * 16;
    const uint64_t nblk = (t.nbuckets + TEXT_T - 1) / TEXT_T;
    if (nblk == 0) return hipSuccess;
    auto kern = k_text_digest<W>;
    hipError_t e = set_smem(kern, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3((unsigned)nblk), dim3(TEXT_T), lds, s, t, count_mode, a, k, out);
    return hipGetLastError();
}

// --------------------------------------------------------------------------------
// k_hll<W>: HyperLogLog registers of a batch's distinct canonical k-mers, the estimate the
// host sizes tables from (kc_estimate_distinct_device + kc_size_table; the reference takes -s
// from its user, main.cpp:134-154).  2^HLL_P registers in LDS: register = the top HLL_P bits of
// the table key's word 0 (a bijective mix of the key; for W >= 2 of its last word and a hash of
// the others), value = 1 + the leading zeros of its other bits; merged into the context's
// registers with atomicMax.  Each workgroup takes one contiguous range of the stream and reads
// its tiles' packed words from a double-buffered LDS stage (as k_p1): the next tile's words are
// loaded while this tile's windows are hashed, so no window waits for HBM (round 6: the
// grid-stride form read every run's words from HBM with dependent loads, 5.2 ms per C4 batch).
// 1024-thread workgroups: the 64 KiB of registers allow two workgroups per CU.
// --------------------------------------------------------------------------------
constexpr int HLL_T = 1024;
template <int W>
constexpr int hll_stage_words() { return HLL_T * run_w<W>() / 32 + W + 3; }
template <int W>
constexpr size_t hll_smem() { return (size_t)HLL_M * 4 + (size_t)hll_stage_words<W>() * 24; }
template <int W>
__global__ __launch_bounds__(HLL_T) void k_hll(PackedView sv, int k, const DevCounters* __restrict__ ctr,
                                               uint32_t* __restrict__ regs, uint64_t pow5_k, uint64_t pow5_km1) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* r = reinterpret_cast<uint32_t*>(smem);
    constexpr int RUNW = run_w<W>(), TW = HLL_T * RUNW, SW = hll_stage_words<W>();
    static_assert(SW <= HLL_T, "one stage word per thread");
    uint64_t* st_pk = reinterpret_cast<uint64_t*>(smem + (size_t)HLL_M * 4);
    uint32_t* st_bk = reinterpret_cast<uint32_t*>(st_pk + 2 * SW);
    const int tid = threadIdx.x;
    for (uint32_t i = tid; i < HLL_M; i += HLL_T) r[i] = 0;
    const uint64_t M = ctr->stream_len;
    const uint64_t per = ((M + gridDim.x - 1) / gridDim.x + TW - 1) / TW * TW;
    const uint64_t lo = min(M, (uint64_t)blockIdx.x * per), hi = min(M, lo + per);
    const uint64_t wlim = M ? ((M - 1) >> 5) + 1 : 0;  // the last word run_windows may read
    // tile t0 reads words (t0 >> 5) - W - 1 .. (t0 + TW) >> 5 (+1) of the stream (run_windows)
    auto stage_word = [&](uint64_t ts, int i, uint64_t& pw, uint32_t& bw) {
        const int64_t w = (int64_t)(ts >> 5) - (W + 1) + i;
        const bool in = w >= 0 && (uint64_t)w <= wlim;
        pw = in ? sv.pk[w] : 0;
        bw = in ? sv.bk[w] : 0;
    };
    if (lo < hi && tid < SW) stage_word(lo, tid, st_pk[tid], st_bk[tid]);
    __syncthreads();
    const RollConst rk = make_roll<W>(k, pow5_k, pow5_km1);
    int par = 0;
    uint32_t nwin = 0;
    for (uint64_t t0 = lo; t0 < hi; t0 += TW) {
        const uint64_t t1 = min(t0 + TW, hi), r0 = t0 + (uint64_t)tid * RUNW;
        const bool nxt = t0 + TW < hi && tid < SW;
        uint64_t npk = 0;
        uint32_t nbk = 0;
        if (nxt) stage_word(t0 + TW, tid, npk, nbk);  // in flight while this tile is hashed
        if (r0 < t1)
            run_windows_src<W, RUNW>(PkStage{st_pk + par * SW, st_bk + par * SW, (int64_t)(t0 >> 5) - (W + 1)}, r0,
                                     t1, rk, [&](int, bool valid, const uint64_t (&fwd)[W], const uint64_t (&rc)[W]) {
                nwin += valid;
                uint64_t key[W], tk[W];
                canonical<W>(fwd, rc, key);
                to_tkey<W>(key, tk);
                const uint32_t j = (uint32_t)(tk[0] >> (64 - HLL_P));
                const uint64_t rest = (tk[0] << HLL_P) | (1ULL << (HLL_P - 1));  // (<= 64 - HLL_P zeros)
                // (no branch: an invalid window merges 0, which changes nothing)
                atomicMax(&r[j], valid ? (uint32_t)__builtin_clzll(rest) + 1 : 0u);
            });
        if (nxt) {
            st_pk[(par ^ 1) * SW + tid] = npk;
            st_bk[(par ^ 1) * SW + tid] = nbk;
        }
        __syncthreads();
        par ^= 1;
    }
    for (uint32_t i = tid; i < HLL_M; i += HLL_T)
        if (r[i]) atomicMax(&regs[i], r[i]);
    block_add4(nwin, 0, 0, 0, &const_cast<DevCounters*>(ctr)->est_windows, nullptr, nullptr, nullptr);
}

// k_hll_s<W> (W <= 4): the same registers over a 2^-HLL_SB sample of the distinct canonical k-mers.
// Every window's canonical key is formed (the rolling extraction) and a cheap strand-symmetric
// hash of it (one 32-bit multiply of its folded halves) picks 1 in 2^HLL_SB distinct keys; only
// those take the table-key mix (the side hash's fmix64s and tmix: 3 to 7 64-bit multiplies) and
// the register update.  A sampled key joins its wave's ring of HLL_Q keys in LDS (ballot + mbcnt
// positions), and whenever 64 wait, every lane of the wave hashes one of them: the expensive half
// runs with all lanes busy on 1/8 of the windows (the unsampled kernel ran it on every window).
// The host scales the estimate by 2^HLL_SB (kc_estimate_distinct_device).  One 1024-thread
// workgroup per CU (registers 64 KiB + rings 16 waves x HLL_Q x W words + the stage).
constexpr int HLL_Q = 128;  // ring entries per wave (a window step adds at most 64)
// windows per thread and run: the run's start (the break scan and the first window's reverse
// complement, O(W)) is paid once per KC_HLL_RUNW windows
#ifndef KC_HLL_RUNW
#define KC_HLL_RUNW 24
#endif
constexpr int HLL_RUNW = KC_HLL_RUNW;
template <int W>
constexpr int hll_s_stage_words() { return HLL_T * HLL_RUNW / 32 + W + 3; }
template <int W>
constexpr size_t hll_s_smem() {
    return (size_t)HLL_M * 4 + (size_t)hll_s_stage_words<W>() * 24 + (size_t)(HLL_T / 64) * HLL_Q * W * 8;
}
template <int W>
__global__ __launch_bounds__(HLL_T) void k_hll_s(PackedView sv, int k, const DevCounters* __restrict__ ctr,
                                                 uint32_t* __restrict__ regs, uint64_t pow5_k, uint64_t pow5_km1) {
    static_assert(hll_sample_bits(W) > 0, "sampled keys of up to four words");
    constexpr int SB = hll_sample_bits(W);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* r = reinterpret_cast<uint32_t*>(smem);
    constexpr int RUNW = HLL_RUNW, TW = HLL_T * RUNW, SW = hll_s_stage_words<W>();
    static_assert(SW <= HLL_T, "one stage word per thread");
    uint64_t* st_pk = reinterpret_cast<uint64_t*>(smem + (size_t)HLL_M * 4);
    uint32_t* st_bk = reinterpret_cast<uint32_t*>(st_pk + 2 * SW);
    const int tid = threadIdx.x, lane = tid & 63;
    uint64_t* ring = reinterpret_cast<uint64_t*>(smem + (size_t)HLL_M * 4 + (size_t)SW * 24) +
                     (size_t)(tid >> 6) * HLL_Q * W;
    for (uint32_t i = tid; i < HLL_M; i += HLL_T) r[i] = 0;
    const uint64_t M = ctr->stream_len;
    const uint64_t per = ((M + gridDim.x - 1) / gridDim.x + TW - 1) / TW * TW;
    const uint64_t lo = min(M, (uint64_t)blockIdx.x * per), hi = min(M, lo + per);
    const uint64_t wlim = M ? ((M - 1) >> 5) + 1 : 0;
    auto stage_word = [&](uint64_t ts, int i, uint64_t& pw, uint32_t& bw) {
        const int64_t w = (int64_t)(ts >> 5) - (W + 1) + i;
        const bool in = w >= 0 && (uint64_t)w <= wlim;
        pw = in ? sv.pk[w] : 0;
        bw = in ? sv.bk[w] : 0;
    };
    if (lo < hi && tid < SW) stage_word(lo, tid, st_pk[tid], st_bk[tid]);
    __syncthreads();
    const RollConst rk = make_roll<W>(k, pow5_k, pow5_km1);
    // ring [head, tail) of the wave's sampled keys (wave-uniform counters)
    uint32_t head = 0, tail = 0;
    // `n` (<= 64) keys from the ring's head, one per lane: the table-key mix and the register
    auto drain = [&](uint32_t n) {
        __builtin_amdgcn_wave_barrier();  // (the ring's stores of other lanes first)
        if (lane < (int)n) {
            const uint32_t e = (head + lane) & (HLL_Q - 1);
            uint64_t key[W], tk[W];
#pragma unroll
            for (int w = 0; w < W; w++) key[w] = ring[e * W + w];
            to_tkey<W>(key, tk);
            const uint32_t j = (uint32_t)(tk[0] >> (64 - HLL_P));
            const uint64_t rest = (tk[0] << HLL_P) | (1ULL << (HLL_P - 1));
            atomicMax(&r[j], (uint32_t)__builtin_clzll(rest) + 1);
        }
        head += n;
    };
    int par = 0;
    uint32_t nwin = 0;
    for (uint64_t t0 = lo; t0 < hi; t0 += TW) {
        const uint64_t t1 = min(t0 + TW, hi), r0 = t0 + (uint64_t)tid * RUNW;
        const bool nxt = t0 + TW < hi && tid < SW;
        uint64_t npk = 0;
        uint32_t nbk = 0;
        if (nxt) stage_word(t0 + TW, tid, npk, nbk);
        // (a thread past the tile's end still takes part in the wave's ballots: run_windows_src
        // reports its windows invalid)
        run_windows_src<W, RUNW>(PkStage{st_pk + par * SW, st_bk + par * SW, (int64_t)(t0 >> 5) - (W + 1)},
                                 r0 < t1 ? r0 : t1, t1, rk,
                                 [&](int, bool valid, const uint64_t (&fwd)[W], const uint64_t (&rc)[W]) {
            nwin += valid;
            uint64_t key[W];
            canonical<W>(fwd, rc, key);
            uint32_t x = (uint32_t)key[W - 1] ^ __builtin_rotateleft32((uint32_t)(key[W - 1] >> 32), 13);
#pragma unroll
            for (int w = 0; w + 1 < W; w++)
                x ^= __builtin_rotateleft32((uint32_t)key[w], 5 + 7 * w) ^
                     __builtin_rotateleft32((uint32_t)(key[w] >> 32), 19 + 3 * w);
            const bool take = valid && ((x * 0x9E3779B1u) >> (32 - SB)) == 0;
            const uint64_t m = __ballot(take);
            if (take) {
                const uint32_t e = (tail + lane_rank(m)) & (HLL_Q - 1);
#pragma unroll
                for (int w = 0; w < W; w++) ring[e * W + w] = key[w];
            }
            tail += (uint32_t)__popcll(m);
            if (tail - head >= 64) drain(64);
        });
        if (nxt) {
            st_pk[(par ^ 1) * SW + tid] = npk;
            st_bk[(par ^ 1) * SW + tid] = nbk;
        }
        __syncthreads();
        par ^= 1;
    }
    drain(tail - head);
    __syncthreads();
    for (uint32_t i = tid; i < HLL_M; i += HLL_T)
        if (r[i]) atomicMax(&regs[i], r[i]);
    block_add4(nwin, 0, 0, 0, &const_cast<DevCounters*>(ctr)->est_windows, nullptr, nullptr, nullptr);
}

template <int W>
hipError_t WOps<W>::hll(PackedView sym, int k, DevCounters* ctr, uint32_t* regs, hipStream_t s) {
    if constexpr (hll_sample_bits(W) > 0) {
        const size_t sm = hll_s_smem<W>();
        hipError_t e = set_smem(k_hll_s<W>, sm);
        if (e != hipSuccess) return e;
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        hipLaunchKernelGGL(k_hll_s<W>, dim3((unsigned)std::max(1, cus)), dim3(HLL_T), sm, s, sym, k, ctr, regs,
                           pow5_mod54(k), pow5_mod54(k - 1));
        return hipGetLastError();
    } else {
        const size_t sm = hll_smem<W>();
        hipError_t e = set_smem(k_hll<W>, sm);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_hll<W>, dim3(512), dim3(HLL_T), sm, s, sym, k, ctr, regs, pow5_mod54(k),
                           pow5_mod54(k - 1));
        return hipGetLastError();
    }
}

}  // namespace kc
