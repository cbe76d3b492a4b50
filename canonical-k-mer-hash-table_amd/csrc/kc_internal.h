// kc_internal.h -- declarations shared by the HIP kernels (kc_tokenize.hip, kc_count.hip) and the
// host side of the C ABI (kc_api.cpp).  Not part of the public boundary
// (that is include/kc_api.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kc_api.h"

namespace kc {

// Staged-batch geometry.  Each reference chunk (text_reader.h:17-36) is placed at a
// TILE-aligned offset of the device stage buffer so that no tile straddles two
// chunks; the tokenizer then works per 4 KiB tile.
constexpr int TILE = 4096;
constexpr int TILE_THREADS = 256;          // 16 bytes per thread
constexpr int COUNT_THREADS = 256;
constexpr int RUN = 32;                    // consecutive symbols rolled per thread
constexpr int BUCKET_WORDS = 16;           // 128-byte buckets
constexpr int BPR = 512;                   // buckets per region: 64 KiB, one LDS-resident table (2^BPR_BITS)
constexpr uint64_t EMPTY = 0;              // empty slot (a stored word 0 is never 0, see kc_common.h)
constexpr int BPR_BITS = 9;
constexpr uint64_t READY = 1ULL << 62;     // multi-word slot published flag, in the count word
constexpr uint64_t CNT_MASK = READY - 1;
constexpr int TEXT_T = 256;                // buckets per workgroup of the text formatter
constexpr int MAX_NH = 10;                 // -f >= 0.001  =>  ceil(-ln f / ln 2) <= 10
constexpr uint8_t SYM_BREAK = 4;
constexpr int BF_BLOCKS_PER_REGION = 1024; // Bloom blocks (64 B) per LDS-resident filter region: 64 KiB
constexpr uint32_t RT_MAX_PARTS = 64;      // shards of the table routing (LDS per-owner counters)
constexpr uint32_t MAX_SEG_GROUP = 128;    // level-2 segments one level-3 workgroup reads (k_p3, k_b3)

// symbol-stream code for byte b outside a header (functions_strings.cpp:56-70)
enum Fmt { FMT_FASTA = 0, FMT_FASTQ = 1, FMT_PLAIN = 2 };

struct ChunkDesc {          // one reference chunk inside the stage buffer
    uint64_t src_off;       // offset in the source image (device-resident path)
    uint64_t stage_off;     // TILE-aligned offset in the stage buffer
    uint64_t len;           // bytes
    uint32_t bh;            // broken_header (text_reader.h:24)
    uint32_t pad;
};

struct TileInfo {           // written by k_tile_summary, consumed by k_tile_scan / k_emit
    uint32_t nl;            // FASTA newlines (removed from the symbol stream)
    uint32_t valid;         // bytes of the chunk inside this tile
    uint8_t marker;         // last header marker: 0 none, 1 '\n', 2 '>'
    uint8_t first;          // tile starts a chunk
    uint8_t bh;             // chunk's broken_header (only meaningful when first)
    uint8_t pad;
    uint32_t avail;         // readable chunk bytes from the tile start (capped at TILE + 64)
    uint64_t src;           // source offset of the tile's first byte
};

struct TileOut {            // written by the tile scan (per tile: block-local; per 1024-tile block: prefix)
    uint64_t out_off;       // first symbol index of the tile in the stream
    uint32_t hs_in;         // header state entering the tile (block-local: transform code)
    uint32_t pad;
};

// Device-side counters (one 128-byte line each to avoid false sharing).
struct DevCounters {
    unsigned long long windows;         uint64_t _p0[15];
    unsigned long long inserted;        uint64_t _p1[15];
    unsigned long long overflow;        uint64_t _p2[15];
    unsigned long long new_in_first;    uint64_t _p3[15];
    unsigned long long new_in_second;   uint64_t _p4[15];
    unsigned long long failed_in_first; uint64_t _p5[15];
    unsigned long long dump_n;          uint64_t _p6[15];
    unsigned long long occupied;        uint64_t _p7[15];
    unsigned long long stream_len;      uint64_t _p8[15];
    unsigned long long bf_windows;      uint64_t _p9[15];
    unsigned long long invalid;         uint64_t _p10[15];  // received keys with word 0 == 0 (skipped)
    unsigned long long part_overflow;   uint64_t _p11[15];  // a fixed-capacity segment overflowed (this batch)
    unsigned long long part_fallbacks;  uint64_t _p12[15];  // batches redone on the exact layout
    // skew (segmented batches): entries of the batch's skew list (keys that did not fit their
    // segment + records of repeated windows), the records among them, and the job totals
    unsigned long long spill_n;         uint64_t _p13[15];
    unsigned long long heavy_n;         uint64_t _p14[15];
    unsigned long long spilled;         uint64_t _p15[15];
    unsigned long long heavy;           uint64_t _p16[15];
    // deferred level 3: a batch's part_overflow held aside while the group's level 3 runs
    unsigned long long held_overflow;   uint64_t _p19[15];
    // the distinct estimate's pass: valid windows (sizes the partition levels of the counting pass that
    // reads its tokenized batches)
    unsigned long long est_windows;     uint64_t _p20[15];
};

// The symbol stream: 32 symbols per word, symbol j of word w at bits 62-2j of pk[w]
// (A=0 C=1 G=2 T=3, big-endian so a window is a contiguous bit range) and break
// flags at bit 31-j of bk[w] (non-ACGT, header byte, chunk start).
struct PackedView {
    uint64_t* pk;
    uint32_t* bk;
};

struct TableView {
    uint64_t* buckets;      // nbuckets * BUCKET_WORDS
    uint64_t nbuckets;      // R * BPR
    uint64_t R;             // regions = F1 * F2 (kc_common.h region_of)
    uint32_t F1, F2;        // partition fan-outs of the two scatter levels (F2 a power of two)
    int f2bits;             // log2 F2
    int W;                  // key words
    int S;                  // slots per bucket
};

// Buffers of the partitioned insert (keys -> coarse bins -> regions -> LDS tables).
struct PartBufs {
    uint32_t nblk1;         // level-1 workgroups (each owns a contiguous symbol range)
    uint32_t B2;            // level-2 workgroups per coarse bin
    uint32_t* hist1;        // [F1][nblk1]
    uint64_t* off1;         // F1*nblk1 + 1 exclusive offsets
    uint32_t* hist2;        // [R][B2]
    uint64_t* off2;         // R*B2 + 1
    uint64_t* bsum;         // scan scratch: one entry per 4096 histogram entries
    uint64_t* keys1;        // coarse-binned keys (W words each)
    uint64_t* keys2;        // region-binned keys
    uint64_t cap1, cap2;    // segmented layout: keys per segment of levels 1 / 2 (0 = exact layout)
    const uint64_t* seg_start;  // level 3 over runs at arbitrary offsets ([R][B2] first items;
                                // nullptr = fixed-capacity segments of cap2)
    uint64_t* spill;        // segmented batches: the skew list ({key words, count} records of keys past
    uint64_t spill_cap;     // a segment's end and of repeated windows; Bloom pass: keys), spill_cap entries
    uint32_t* keep_fill;    // Bloom pass keeping its partitions (partition reuse): copies of the
    uint32_t* keep_fill2;   // segment fills of levels 1 and 2 (the skew-list pass reuses hist1/2)
    int rec6;               // segmented count pass, one-word keys, R >= 2^16: level 2 writes 6-byte
                            // records (kc_count_impl.h StoreRec6) that its level 3 reads
    // two-word keys in power-of-two bin geometries (the Bloom pass that keeps its partitions, and
    // the counting pass from them): 12-byte level records (kc_count_impl.h Rec12).  rec12 bits:
    // R12_P1 k_p1 writes them at level 1, R12_IN k_p2f reads level 1 as them, R12_OUT k_p2f
    // writes them at level 2, R12_L2 k_b3 / k_p3 read level 2 as them
    int rec12;
    int r12_hb;             // bits of table-key word 1 above 32 (2k - 96, or 0)
    int r12_xb1, r12_xb2;   // bits of t0's top half below the level-1 / level-2 bin
    int r12_b2s;            // log2 of the level-2 segments per bin (fine bin of a segment = segment >> r12_b2s)
    // kc_route_hint: every level-3 workgroup (k_p3) also writes its region's record counts per
    // owner shard for the two 256-bucket blocks of kc_route_table_device ([own_parts][own_nblk];
    // own_parts = 0: off), so the route of a table counted by level 3 skips its count pass
    uint32_t* own_hist;
    uint32_t own_parts;
    uint64_t own_nblk;
    // deferred level 3 (kc_api.cpp run_batch): the level-2 segments of several batches of one image
    // stay in keys2 and one level-3 pass inserts them all, i.e. one sweep of the table per group of
    // batches instead of per batch.  Level 2 writes segment r * b2t + b2off + j of region r (b2t = 0:
    // B2 and no offset, one batch); the deferred level 3 runs with B2 = b2t.
    uint32_t b2t;
    uint32_t b2off;
    // a later batch of a deferred group: its skew-list entries go after the group's earlier
    // batches' (the list is inserted once, after the group's level 3: kc_api.cpp run_deferred)
    uint32_t keep_skew;
};
constexpr int R12_P1 = 1, R12_IN = 2, R12_OUT = 4, R12_L2 = 8;
// R12_REG: the records are in the table's own geometry (the counting pass's levels): a bin's
// lowest x is region_xlo of its first region, not bin << xb
constexpr int R12_REG = 16;
// bits that hold every value of a span (ceil(log2(span)), at most 32)
inline int span_bits32(uint64_t span) {
    int b = 0;
    while (b < 32 && (1ULL << b) < span) b++;
    return b;
}
// the level-2 record of the counting pass in a table of R regions (kc_count_impl.h
// launch_part_w): 6 bytes for one-word keys once R >= 2^16 (StoreRec6), 12 for two-word keys
// whose region spans few enough values of x (Rec12: hb + 1 + xb2 <= 32), else the W key words
inline uint64_t level2_record_bytes(int W, int k, uint64_t R) {
    if (W == 1) return R >= (1ULL << 16) ? 6 : 8;
    if (W == 2 && R) {
        const int hb = 2 * k - 96 > 0 ? 2 * k - 96 : 0;
        if (hb + 1 + span_bits32(((1ULL << 32) + R - 1) / R) <= 32) return 12;
    }
    return 8ull * (uint64_t)W;
}

struct BloomView {
    uint32_t* bits;         // 2 * nbits filter bits, interleaved: bit 2h = filter 1, 2h+1 = filter 2
    uint64_t mask;          // nbits - 1
    int nh;                 // ceil(hf): pass-1 hashes
    int nh_gate;            // trunc(hf): pass-2 gate hashes
    int blocked;            // 1: one 512-bit block per k-mer (kc_count.hip, blocked layout)
    uint64_t nblocks;       // blocks (a power of two: max(1, nbits / 256))
    uint32_t slice_blocks;  // gated level 3: LDS capacity for a table region's filter-2 slice
                            // (blocks; 0 = the gate reads HBM)
};

constexpr int MAX_K = 479;     // largest k: fifteen key words + the count fill one 128-byte bucket
constexpr int MAX_W = 15;      // (KCO_MAXW of the oracle)
inline int words_for_k(int k) { return k / 32 + 1; }          // spare top bit for EMPTY
inline int slots_per_bucket(int W) { return BUCKET_WORDS / (W + 1); }

// Windows rolled per thread in the partitioned kernels, and the workgroup size of the
// segmented level 1 (tile = threads x windows), by key width: wide keys take fewer
// windows per thread and smaller groups so that the registers and the LDS tile fit.
constexpr int run_width(int W) { return W == 1 ? 16 : W == 2 ? 8 : W <= 4 ? 8 : 4; }
// The segmented level 1 (k_p1) of one- to four-word keys: 512-thread workgroups, two per CU.
// (1024 threads with half the windows per thread -- 8 waves per SIMD within 64 VGPRs -- spill
// and ran 30 % slower: profiles/r03_ab_p1_nt.txt)
constexpr int scatter_threads_w(int W) { return W <= 4 ? 512 : 256; }
constexpr int p1_runw(int W) { return run_width(W); }
constexpr int p1_tile(int W) { return scatter_threads_w(W) * p1_runw(W); }  // windows per segmented level-1 tile
// level 2 (k_p2f): workgroup size by key width, and its LDS for F2 regions per coarse bin
// a scatter's per-bin LDS arrays (k_count_impl.h PartLds: 4 x u32 + 1 x u64 per bin, the
// tile's keys after them at a 16-byte boundary) and its static extras
constexpr size_t bin_lds_bytes(uint32_t F) { return ((size_t)F * 24 + 15) / 16 * 16 + 16; }
constexpr int p2f_threads_w(int W) { return W <= 2 ? 1024 : W <= 4 ? 512 : 256; }
// k_p1's LDS stage of the packed stream: two buffers of the words one tile reads, 12 bytes each
constexpr size_t p1_stage_bytes(int W) { return (size_t)(p1_tile(W) / 32 + W + 3) * 24; }
// segmented level 1 (k_p1, W-word output keys + the heavy table + the stage) for F1 coarse bins
constexpr size_t p1_lds_bytes(int W, uint32_t F1) {
    return bin_lds_bytes(F1) + (size_t)p1_tile(W) * 8 * W + (size_t)64 * (W + 1) * 8 + p1_stage_bytes(W);
}
// nt: the level-2 workgroup (0 = p2f_threads_w; wide keys fall back to half of it when their
// table's F2 does not fit beside the full tile, k_count_impl.h launch_p2f)
constexpr size_t p2f_lds_bytes(int W, uint32_t F2, uint32_t nseg, int nt = 0) {
    return bin_lds_bytes(F2) + (size_t)(nt ? nt : p2f_threads_w(W)) * run_width(W) * 8 * W + ((size_t)nseg + 1) * 4;
}
constexpr size_t LDS_BYTES = 160 * 1024;  // per CU (one workgroup may take all of it)
// Big tables (the whole C4 job on one GPU: 525 coarse bins) leave the 4096-window tile of the
// two-word level 1 runs of fewer than 8 keys per bin, and the launcher then keeps one 512-thread
// workgroup per CU (8 waves) so that L2 merges the partial lines.  Two-word keys take a
// 1024-thread level 1 instead (one workgroup per CU, 16 waves, 128 VGPRs): an 8192-window
// tile, runs twice as long, when its LDS fits beside the bins.
constexpr int P1_WIDE_THREADS = 1024;
constexpr size_t p1_lds_bytes_nt(int W, uint32_t F1, int nt) {
    return bin_lds_bytes(F1) + (size_t)nt * p1_runw(W) * 8 * W + (size_t)64 * (W + 1) * 8 +
           (size_t)(nt * p1_runw(W) / 32 + W + 3) * 24;
}
constexpr bool p1_wide(int W, uint32_t F1) {
    return W == 2 && (uint64_t)p1_tile(W) < 8ULL * F1 && p1_lds_bytes_nt(W, F1, P1_WIDE_THREADS) <= LDS_BYTES;
}
// the largest level-1 tile a table pass of W-word keys may run (the host's segment sizing rounds
// block ranges to it)
constexpr int p1_tile_max(int W) { return W == 2 ? P1_WIDE_THREADS * p1_runw(W) : p1_tile(W); }

// ---- launchers (kc_tokenize.hip, kc_count.hip) -------------------------------------------------
// src: bytes the chunk descriptors' src_off point into (host stage or device image)
hipError_t launch_tokenize(const uint8_t* src, uint64_t ntiles, const ChunkDesc* d_chunks, int n_chunks,
                           int fmt, TileInfo* tiles, TileOut* touts, TileOut* tblk, PackedView sv,
                           uint64_t sym_bound, DevCounters* ctr, hipStream_t s);
// mode: 0 count all windows, 1 Bloom pass 1, 2 count windows passing the Bloom gate
hipError_t launch_count(PackedView sv, uint64_t sym_bound, int k, int mode, TableView t, BloomView bf,
                        DevCounters* ctr, hipStream_t s);
// partitioned insert for modes 0 and 2 (same table, same result as launch_count; mode 2
// gates at level 3 on the blocked Bloom layout, at level 1 on the reference layout)
// fresh: the table is all zero (just allocated or reset): level 3 does not read it
// phase (segmented layout): bit 0 = the single-pass levels (PH_MAIN), bit 1 = the batch's
// tail: the skew list, the batch's bookkeeping and the exact pipeline behind the device
// overflow gate (PH_TAIL).  The host may run the tail only when the main phase left a skew
// list or an overflow (kc_api.cpp); with both empty every tail kernel is a no-op.
constexpr int PH_MAIN = 1, PH_TAIL = 2, PH_ALL = 3;
// Counting pass, deferred level 3 (segmented layout): the batch's levels 1-2 into its slot of the
// group's level-2 segments (PartBufs b2t / b2off), and level 3 over the whole group (pb.B2 = b2t)
constexpr int PH_L12 = 16, PH_L3 = 32;
hipError_t launch_count_partitioned(PackedView sv, uint64_t sym_bound, int k, int mode, TableView t,
                                    BloomView bf, DevCounters* ctr, PartBufs pb, int fresh, hipStream_t s,
                                    int phase = PH_ALL);
// Bloom pass 1 on the blocked layout, partitioned: ft = the filter's region geometry
// (R = filter regions of nblocks / R <= 1024 blocks, F1 x F2 as for the table; no buckets);
// fresh: the filter is all zero (level 3 does not read it)
// keep: levels 1 and 2 move whole table keys in the fine geometry fg (kept for the counting
// pass, count_reuse); otherwise fg is unused
hipError_t launch_bloom_partitioned(PackedView sv, int k, int W, BloomView bf, TableView ft, TableView fg,
                                    DevCounters* ctr, PartBufs pb, int fresh, int keep, hipStream_t s,
                                    int phase = PH_ALL);
// the counting pass from the partitions kept by the Bloom pass (pb: their buffers), from
// level 2 (level 2) or level 1 (level 1); gate: behind the Bloom gate (0: -m 1 -b, whose
// filter is ignored); windows: the batch's windows (counted by the Bloom pass)
hipError_t launch_count_reuse(int W, TableView t, BloomView bf, DevCounters* ctr, PartBufs pb, int fresh, int level,
                              int gate, uint64_t windows, hipStream_t s);
// The two passes over pre-aggregated {W key words, count} records (the owner side of the sharded
// Bloom filter, kaarme_amd/sharded.py): Bloom pass 1 (a record of count >= 2 inserted twice) into
// the filter's regions ft, and the gated (gate = 1) or plain counting pass into the table t.
// pb: exact-layout buffers for items of W + 1 words (kc_api.cpp ensure_part_geo)
hipError_t launch_bloom_records(int W, const uint64_t* rec, uint64_t n, BloomView bf, TableView ft, DevCounters* ctr,
                                PartBufs pb, int fresh, hipStream_t s);
hipError_t launch_count_records(int W, const uint64_t* rec, uint64_t n, TableView t, BloomView bf, DevCounters* ctr,
                                PartBufs pb, int fresh, int gate, hipStream_t s);
// deferred level 3: part_overflow -> held_overflow (and cleared), or back (restore)
hipError_t launch_hold_overflow(DevCounters* ctr, int restore, hipStream_t s);
// 64-bit checksum of the chunks' bytes (a promise check between two passes over one image):
// CHECKSUM_SLOTS partial sums in out (their sum is the checksum)
constexpr int CHECKSUM_SLOTS = 64;
hipError_t launch_checksum(const uint8_t* src, const ChunkDesc* d_chunks, int n_chunks, uint64_t max_len,
                           unsigned long long* out, hipStream_t s);
// sharded Bloom filter: combine nparts copies (consecutive, n words each) of one word range of
// the filter into out -- filter 1 = OR, filter 2 = OR | (filter-1 bits set in >= 2 copies);
// blocked: the range starts at a block (16 words); else the reference's 2h / 2h+1 bit pairs
hipError_t launch_bloom_merge(const uint32_t* parts, uint32_t nparts, uint64_t n, int blocked, uint32_t* out,
                              hipStream_t s);
// set filter-2 bits of the whole filter: CHECKSUM_SLOTS partial sums in out
hipError_t launch_bloom_popcount2(const uint32_t* words, uint64_t n, int blocked, unsigned long long* out,
                                  hipStream_t s);
// hash-prefix sharding: windows -> table keys grouped by owner (offsets in pb.off1)
hipError_t launch_route(PackedView sym, int k, int W, DevCounters* ctr, PartBufs pb, uint32_t parts, uint64_t* out,
                        hipStream_t s);
// insert an array of table keys into this shard's table
hipError_t launch_insert_keys(const uint64_t* keys, uint64_t n, bool partitioned, TableView t, DevCounters* ctr,
                              PartBufs pb, int fresh, hipStream_t s);
// pre-aggregated sharding: out == nullptr -> per-(owner, block) record counts into hist and
// their exclusive scan into off (off[parts * nblk] = total); else scatter the records
// out == nullptr: the count pass (per-block record counts into hist, skipped when hist_ready:
// the counting passes kept them, kc_route_hint) and their scan; else the scatter into out
hipError_t launch_route_table(TableView t, uint32_t parts, uint32_t* hist, uint64_t* off, uint64_t* bsum,
                              uint64_t* out, hipStream_t s, int hist_ready = 0);
hipError_t launch_insert_counts(const uint64_t* rec, uint64_t n, bool partitioned, TableView t, DevCounters* ctr,
                                PartBufs pb, int fresh, hipStream_t s);
// shard merge of records that arrive as G groups each sorted by this table's region
// (kc_route_table_device order on a table of the same geometry): gstart[G+1] group
// offsets (device).  check: flag |= 1 if some group is not sorted.  runs: region run
// bounds per group (m_start [(R+1)][G], m_len [R][G]) and one level-3 pass over them.
hipError_t launch_check_runs(const uint64_t* rec, const uint64_t* gstart, uint32_t G, uint64_t maxn, TableView t,
                             unsigned long long* flag, hipStream_t s);
hipError_t launch_insert_counts_runs(const uint64_t* rec, const uint64_t* gstart, uint32_t G, TableView t,
                                     DevCounters* ctr, uint32_t* m_len, uint64_t* m_start, int fresh, hipStream_t s);
// HyperLogLog registers of the distinct-count estimate (kc_count_impl.h k_hll)
constexpr int HLL_P = 14;
constexpr uint32_t HLL_M = 1u << HLL_P;
// k_hll of keys up to four words hashes a 2^-HLL_SB sample of the distinct k-mers (a cheap
// strand-symmetric hash of the canonical key picks them): the estimate is 2^HLL_SB x the sample's
constexpr int hll_sample_bits(int W) { return W <= 4 ? 3 : 0; }
hipError_t launch_hll(PackedView sym, int k, int W, DevCounters* ctr, uint32_t* regs, hipStream_t s);
// Super-k-mer routing of a tokenized batch to nshards owners by canonical minimizer (kc_skm.hip):
// per owner a packed symbol stream (out_pk / out_bk regions of cap words), cursor[] = words used,
// wins[] = windows routed, *ovf = 1 if a region overflowed
constexpr uint32_t SKM_MAX_SHARDS = 64;
constexpr int SKM_DEFAULT_M = 15;  // minimizer length (odd: no palindromic m-mers); min(15, k)
// the m-mer order: h(x) = fmix32(lo32(x) ^ hi32(x) * SKM_FOLD ^ SKM_SEED32) (a bijection for m <= 16)
constexpr uint32_t SKM_SEED32 = 0x4C957F2Du, SKM_FOLD = 0x9E3779B1u;
hipError_t launch_skm_route(PackedView sv, const DevCounters* ctr, uint64_t sym_bound, int k, int m, uint32_t nshards,
                            uint64_t* out_pk, uint32_t* out_bk, uint64_t cap, unsigned long long* cursor,
                            unsigned long long* wins, unsigned long long* ovf, hipStream_t s);
hipError_t launch_dump(TableView t, int count_mode, uint64_t min_abundance, uint64_t* out, DevCounters* ctr,
                       hipStream_t s);
// GPU text formatting (kc_write): bytes of each TEXT_T-bucket block into block_bytes and
// their exclusive scan into off (off[nblocks] = total; bsum: (nblocks + 4095) / 4096 + 2
// words of scratch); then k_text for blocks [blk0, blk0 + nblk) into out (offset base),
// lds >= the largest of those blocks' bytes
hipError_t launch_text_bytes(TableView t, int count_mode, uint64_t a, int k, uint32_t* block_bytes, uint64_t* off,
                             uint64_t* bsum, hipStream_t s);
hipError_t launch_text(TableView t, int count_mode, uint64_t a, int k, uint64_t blk0, uint64_t nblk,
                       const uint64_t* off, uint64_t base, uint8_t* out, size_t lds, hipStream_t s);
// order-independent digest of those lines (kc_output_digest): out[4] += {lines, sum T(c), sum of
// XXH64(line), xor of XXH64(line)} (out zeroed by the caller)
hipError_t launch_text_digest(TableView t, int count_mode, uint64_t a, int k, unsigned long long* out, hipStream_t s);
hipError_t launch_xxh64(const uint64_t* v, const uint64_t* seed, uint64_t n, uint64_t* out, hipStream_t s);
hipError_t launch_synth(uint8_t* dst, uint64_t first_read, uint64_t n_reads, uint64_t seed, uint64_t genome_len,
                        uint32_t read_len, uint32_t wrap, double err_rate, double n_rate, const kc_synth_skew* skew,
                        hipStream_t s);

// ---- per-key-width entry points (kc_count_impl.h, one translation unit per W) ------------------
template <int W>
struct WOps {
    static hipError_t count(PackedView sym, uint64_t sym_bound, int k, int mode, TableView t, BloomView bf,
                            DevCounters* ctr, hipStream_t s);
    static hipError_t count_partitioned(PackedView sym, int k, int mode, TableView t, BloomView bf, DevCounters* ctr,
                                        PartBufs pb, int fresh, hipStream_t s, int phase);
    static hipError_t bloom_partitioned(PackedView sym, int k, BloomView bf, TableView ft, TableView fg,
                                        DevCounters* ctr, PartBufs pb, int fresh, int keep, hipStream_t s, int phase);
    static hipError_t count_reuse(TableView t, BloomView bf, DevCounters* ctr, PartBufs pb, int fresh, int level,
                                  int gate, uint64_t windows, hipStream_t s);
    static hipError_t bloom_records(const uint64_t* rec, uint64_t n, BloomView bf, TableView ft, DevCounters* ctr,
                                    PartBufs pb, int fresh, hipStream_t s);
    static hipError_t count_records(const uint64_t* rec, uint64_t n, TableView t, BloomView bf, DevCounters* ctr,
                                    PartBufs pb, int fresh, int gate, hipStream_t s);
    static hipError_t route(PackedView sym, int k, DevCounters* ctr, PartBufs pb, uint32_t parts, uint64_t* out,
                            hipStream_t s);
    static hipError_t insert_keys(const uint64_t* keys, uint64_t n, bool partitioned, TableView t, DevCounters* ctr,
                                  PartBufs pb, int fresh, hipStream_t s);
    static hipError_t route_table(TableView t, uint32_t parts, uint32_t* hist, uint64_t* off, uint64_t* bsum,
                                  uint64_t* out, hipStream_t s, int hist_ready);
    static hipError_t insert_counts(const uint64_t* rec, uint64_t n, bool partitioned, TableView t, DevCounters* ctr,
                                    PartBufs pb, int fresh, hipStream_t s);
    static hipError_t check_runs(const uint64_t* rec, const uint64_t* gstart, uint32_t G, uint64_t maxn, TableView t,
                                 unsigned long long* flag, hipStream_t s);
    static hipError_t insert_counts_runs(const uint64_t* rec, const uint64_t* gstart, uint32_t G, TableView t,
                                         DevCounters* ctr, uint32_t* m_len, uint64_t* m_start, int fresh, hipStream_t s);
    static hipError_t dump(TableView t, int count_mode, uint64_t min_abundance, uint64_t* out, DevCounters* ctr,
                           hipStream_t s);
    static hipError_t hll(PackedView sym, int k, DevCounters* ctr, uint32_t* regs, hipStream_t s);
    static hipError_t text_bytes(TableView t, int count_mode, uint64_t a, int k, uint32_t* block_bytes, uint64_t* off,
                                 uint64_t* bsum, hipStream_t s);
    static hipError_t text(TableView t, int count_mode, uint64_t a, int k, uint64_t blk0, uint64_t nblk,
                           const uint64_t* off, uint64_t base, uint8_t* out, size_t lds, hipStream_t s);
    static hipError_t text_digest(TableView t, int count_mode, uint64_t a, int k, unsigned long long* out,
                                  hipStream_t s);
};
// Kaarme's compact representation, built after counting (kc_compact_impl.h)
struct CompactView {
    uint64_t* words;               // nslots 8-byte slot words (kmer.hpp:103-149 layout)
    uint64_t nslots;
    uint64_t* src;                 // build only: full-table slot (bucket * S + s) per compact slot, ~0 = empty
    uint64_t* second;              // chain-start keys, W words each
    unsigned long long* n_second;  // chain starts written
    uint64_t* inv;                 // build only: compact slot per full-table slot (written for occupied ones)
};
template <int W>
struct CompactOps {
    static hipError_t build(TableView t, CompactView c, int k, hipStream_t s);
    static hipError_t dump(CompactView c, int k, uint64_t a, uint64_t* out, unsigned long long* cursor,
                           unsigned long long* stats, hipStream_t s);
    static hipError_t lookup(CompactView c, int k, const uint64_t* keys, uint64_t n, uint32_t* counts, hipStream_t s);
};
hipError_t launch_compact_build(TableView t, CompactView c, int k, hipStream_t s);
// records {W key words, T(c)} of the slots with T(c) >= a (out == nullptr: count into cursor);
// stats[0] += hops, stats[1] = max hops, stats[2] += walks that did not end
hipError_t launch_compact_dump(int W, CompactView c, int k, uint64_t a, uint64_t* out, unsigned long long* cursor,
                               unsigned long long* stats, hipStream_t s);
hipError_t launch_compact_lookup(int W, CompactView c, int k, const uint64_t* keys, uint64_t n, uint32_t* counts,
                                 hipStream_t s);

extern template struct WOps<1>;
extern template struct WOps<2>;
extern template struct WOps<3>;
extern template struct WOps<4>;
extern template struct WOps<5>;
extern template struct WOps<6>;
extern template struct WOps<7>;
extern template struct WOps<8>;
extern template struct CompactOps<1>;
extern template struct CompactOps<2>;
extern template struct CompactOps<3>;
extern template struct CompactOps<4>;
extern template struct CompactOps<5>;
extern template struct CompactOps<6>;
extern template struct CompactOps<7>;
extern template struct CompactOps<8>;

}  // namespace kc
