// kc_api.cpp -- host side of the C ABI (include/kc_api.h): context, staging,
// batch scheduling, table/Bloom sizing and result extraction.  Compiled by hipcc
// into libkc.so together with kc_device.hip.
//
// Data flow per batch (the reference's io_worker -> in_queue -> string_worker,
// parallel_parser.hpp:1230-1519, re-shaped for one device):
//   host chunk -> pinned stage image (chunk at a 4 KiB-aligned offset)
//   -> one async H2D per batch -> tokenize (3 kernels) -> count/bloom kernel.
// Two pinned stage buffers alternate so the host fills one while the device
// consumes the other.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kc_api.h"
#include "kc_internal.h"
#include "kc_synth.h"

using namespace kc;

namespace {

thread_local std::string g_create_error;

constexpr uint64_t kDefaultBatch = 256ull << 20;

uint64_t round_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

}  // namespace

// entries the histogram / offset arrays of one PartBufs were allocated for
struct PartCap {
    uint64_t h1 = 0;  // hist1 entries (off1: h1 + 1)
    uint64_t h2 = 0;  // hist2 entries (off2: h2 + 1)
    uint64_t bs = 0;  // bsum entries
};

struct kc_ctx {
    kc_config cfg{};
    int W = 1, S = 8;
    hipStream_t stream = nullptr;
    std::string err;

    // staging
    uint64_t batch_bytes = 0;
    uint64_t max_chunks = 0;
    uint8_t* h_stage[2] = {nullptr, nullptr};
    ChunkDesc* h_desc[2] = {nullptr, nullptr};
    hipEvent_t h_free[2] = {nullptr, nullptr};  // recorded after the H2D reading buffer i
    hipEvent_t xev = nullptr;                   // orders the context stream with a caller stream
    hipStream_t aux = nullptr;                  // the kept Bloom batch's checksum, beside its levels
    hipEvent_t aev[2] = {nullptr, nullptr};     // caller stream -> aux -> caller stream
    int cur = 0;
    uint64_t cur_used = 0;                      // stage bytes used in h_stage[cur]
    uint64_t cur_n = 0;                         // chunks in h_stage[cur]
    int cur_fmt = -1;
    int cur_pass = -1;                          // 0 count, 1 bloom

    uint8_t* d_stage = nullptr;
    uint64_t* d_pk = nullptr;  // packed symbol stream
    uint32_t* d_bk = nullptr;  // break bitmap
    TileInfo* d_tiles = nullptr;
    TileOut* d_touts = nullptr;
    TileOut* d_tblk = nullptr;  // per-1024-tile block prefixes
    ChunkDesc* d_chunks = nullptr;
    DevCounters* d_ctr = nullptr;

    // table
    uint64_t* d_table = nullptr;
    uint64_t table_cap_bytes = 0;  // allocation size (a Bloom job re-sizes the table per pass)
    uint64_t nbuckets = 0;
    uint64_t R = 0;
    uint32_t F1 = 1, F2 = 1;
    int f2bits = 0;
    bool seg_ok = true;  // the table's geometry fits the segmented single-pass levels (else exact layout)

    // partitioned insert buffers (pb: the table's levels; pbf: the Bloom pass's, same key
    // buffers, own histograms)
    PartBufs pb{}, pbf{};
    PartCap pb_cap{}, pbf_cap{};
    uint64_t* d_keys1 = nullptr;
    uint64_t* d_keys2 = nullptr;
    uint64_t k1_words = 0, k2_words = 0;  // u64 words the level-1 / level-2 key buffers hold
    uint64_t* d_spill = nullptr;           // skew list of a segmented batch (ensure_part_geo)
    uint64_t spill_words = 0;
    bool table_fresh = false;  // the table is all zero (allocated / reset, nothing inserted since)
    uint64_t min_slots = 0;        // the job's -s (or 2 * new_in_second): the reference's table size
    bool strict_capacity = false;  // KC_STRICT_CAPACITY=1: fail past the reference's capacity
    // kc_reset defers the table memset: a fresh level-3 pass writes every region anyway;
    // any other use of the table zeroes it first (materialize_zero)
    bool table_zero_pending = false;
    // kc_route_table_device: per-(owner, block) record counts, their scan, scan scratch
    uint32_t* d_rhist = nullptr;
    uint64_t* d_roff = nullptr;
    uint64_t* d_rbsum = nullptr;
    uint64_t r_cap = 0;
    // kc_route_hint: the level-3 passes keep d_rhist for own_parts owners (PartBufs.own_hist);
    // own_valid = it holds the table's current per-block record counts
    uint32_t own_parts = 0;
    bool own_valid = false;
    uint64_t route_counts_kept = 0;  // kc_route_table_device calls that skipped the count pass
    // kc_insert_counts_runs_device: group offsets, region run starts / lengths
    uint64_t* d_gstart = nullptr;
    uint64_t* d_mstart = nullptr;
    uint32_t* d_mlen = nullptr;
    uint64_t m_cap = 0;  // entries of d_mstart

    // bloom
    uint32_t* d_bloom = nullptr;
    uint64_t bf_bits = 0;
    int nh = 0, nh_gate = 0;
    int bloom_blocked = 1;  // KC_BLOOM_LAYOUT=reference: the reference's independent positions
    bool bloom_final = false;
    bool bloom_fresh = false;  // the filter is all zero (allocated / reset, nothing inserted since)
    TableView bgeo{};          // blocked layout: the filter's region geometry (k_b3 regions)

    // Level-1 reuse (device path): a Bloom job whose Bloom pass is ONE batch over a device
    // image keeps that pass's level-1 output (whole table keys in the filter's coarse bins,
    // launch_bloom_partitioned keep); the table is then sized with the same coarse bins, and
    // a counting pass over the same image and chunks (checked: pointer, chunk list, format
    // and a checksum of the bytes) starts at level 2 instead of tokenizing and extracting
    // every window again (launch_count_reuse).  KC_REUSE=0 disables it.
    int bloom_batches = 0;            // Bloom-pass batches since the job started
    bool reuse_kept = false;          // the (only) Bloom batch kept its level-1 output
    bool reuse_ok = false;            // kc_bloom_finalize: kept, no skew entries, geometry fits
    const uint8_t* reuse_img = nullptr;
    std::vector<ChunkDesc> reuse_chunks;
    int reuse_fmt = -1;
    uint64_t reuse_used = 0;          // stage bytes of the batch
    unsigned long long reuse_sum = 0; // checksum of the Bloom pass's chunk bytes
    uint64_t reuse_windows = 0;       // windows of that batch
    unsigned long long* d_sum = nullptr;  // CHECKSUM_SLOTS partial sums (+ CHECKSUM_SLOTS for kc_bloom_estimate)
    // the counting pass's checksum of its bytes, copied back on the aux stream: context memory, so
    // a call that returns before waiting for that copy leaves it no dangling destination
    unsigned long long h_part[CHECKSUM_SLOTS] = {};
    uint32_t* d_hll = nullptr;            // HLL_M registers of kc_estimate_distinct_device
    // compact representation (kc_compact): slot words, chain-start keys, counters
    uint64_t* d_cwords = nullptr;
    uint64_t cslots = 0;
    uint64_t* d_csecond = nullptr;
    uint64_t cstarts = 0, ckmers = 0;
    unsigned long long* d_cstat = nullptr;  // [0] chain starts / record cursor, [1] hops, [2] max hops, [3] bad walks
    uint32_t* d_keep_fill = nullptr;      // the kept partitions' segment fills: level 1 [F1][nblk1]
    uint32_t* d_keep_fill2 = nullptr;     // and level 2 [R_fine][B2]
    uint64_t keep_fill_cap = 0, keep_fill2_cap = 0;
    TableView fgeo{};                     // the kept partitions' fine geometry (powers of two)
    uint64_t fgeo_max_R = 0;              // the create-time fine regions (the most the LDS fits)
    uint64_t fgeo_next_R = 0;             // fine regions learned from the last finalize (0 = keep)
    int reuse_level = 0;                  // kc_bloom_finalize: 2 = from level 2, 1 = from level 1
    uint64_t reuse_hits = 0;          // counting passes that reused (kc_stats.reused_passes)
    int reuse_last_level = 0;         // the level the last reused pass started from (kc_stats.reuse_level)

    uint64_t n_chunks = 0, n_bytes = 0;

    // Deferred level 3 (device_pass / run_deferred): a counting pass over an image of several
    // batches keeps the level-2 segments of up to defer_g batches in keys2 and inserts them with one
    // level-3 pass -- one sweep of the table per group instead of per batch
    bool defer_on = false;     // the current device_pass defers (set per pass)
    bool defer_last = false;   // the batch being launched is the pass's last
    uint32_t defer_g = 0;      // batches per group
    uint32_t defer_n = 0;      // batches of the current group whose segments wait
    uint64_t skew_prev = 0;    // the group's skew list after its last batch (entries, of them records of
    uint64_t heavy_prev = 0;   // repeated windows): what a batch that overflows leaves to insert
    uint64_t defer_syms = 0;   // the group's segment geometry is sized for batches of this bound
    uint64_t defer_groups = 0; // level-3 passes the deferral ran (kc_stats)
    // super-k-mer routing (kc_route_superkmers_device): the pass-4 batches' parameters and the
    // device cursors [0, 64) words per owner, [64, 128) windows per owner, [128] overflow flag
    unsigned long long* d_skm = nullptr;
    uint32_t skm_shards = 0;
    int skm_m = 0;
    uint64_t* skm_pk = nullptr;
    uint32_t* skm_bk = nullptr;
    uint64_t skm_cap = 0;
    // kc_estimate_distinct_device keeps its tokenized batches for the next counting pass over the
    // same image, chunks and format (kept_*): keep_pk / keep_bk hold batch i's stream at word kept[i].first
    uint64_t* keep_pk = nullptr;
    uint32_t* keep_bk = nullptr;
    uint64_t keep_cap = 0, keep_woff = 0;  // words allocated / used
    bool keep_target = false;              // the estimate pass writes its streams there
    bool kept_valid = false;
    const uint8_t* kept_img = nullptr;
    int kept_fmt = -1;
    std::vector<kc_chunk> kept_chunks;
    std::vector<std::pair<uint64_t, uint64_t>> kept;  // per batch: first word, symbol bound
    uint64_t* d_kept_len = nullptr;                    // per batch: the stream length the tokenizer left
    uint64_t* d_kept_win = nullptr;                    // per batch: the estimate pass's windows so far
    uint64_t kept_len_cap = 0;
    double kept_density = 1.0;                         // the kept batches' largest windows per symbol
    // windows per symbol of the batches being planned (1: tokenized input, where every symbol can
    // end a window; a received super-k-mer stream carries k symbols of context per run)
    double win_density = 1.0;
    // a counting pass failed after some of its batches were counted (a deferred group whose level 3
    // never ran, a failed launch): the table no longer matches the windows counted, so every call
    // that counts or reads the table fails until kc_reset
    std::string broken;

    // profiling: event quadruples {start, after gather, after tokenize, after count}
    bool profiling = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::array<hipEvent_t, 4>> ev_pending;
    kc_timing timing{};
    uint64_t* d_stream_len_probe = nullptr;
    std::vector<uint64_t> pending_symbols_bound;

    hipEvent_t get_event() {
        if (!ev_pool.empty()) {
            hipEvent_t e = ev_pool.back();
            ev_pool.pop_back();
            return e;
        }
        hipEvent_t e = nullptr;
        (void)hipEventCreate(&e);
        return e;
    }

    int fail(int code, const std::string& m) {
        err = m;
        return code;
    }
    int hipfail(hipError_t e, const char* what) {
        err = std::string(what) + ": " + hipGetErrorString(e);
        return KC_ERR_HIP;
    }
};

#define HIPCHK(ctx, expr)                                  \
    do {                                                   \
        hipError_t _e = (expr);                            \
        if (_e != hipSuccess) return (ctx)->hipfail(_e, #expr); \
    } while (0)

// the calls that count into or read the table refuse a job a failed pass left incomplete
#define JOB_OK(ctx)                                                                            \
    do {                                                                                       \
        if (!(ctx)->broken.empty()) return (ctx)->fail(KC_ERR_STATE, (ctx)->broken + " (kc_reset first)"); \
    } while (0)

// ------------------------------------------------------------------------------
// sizing helpers
// ------------------------------------------------------------------------------
static void bloom_sizes(uint64_t U, double fpr, uint64_t* bits, int* nh, int* nh_gate) {
    // main.cpp:402-418: bits = next pow2 >= -U ln f / ln^2 2 (compared as uint64),
    // hf = bits_min / U * ln 2; pass 1 uses ceil(hf) (main.cpp:417), the pass-2 gate
    // receives hf through a uint64_t parameter, i.e. trunc(hf) (parallel_parser.hpp:2397).
    double bits_min = (-double(U) * std::log(fpr)) / std::pow(std::log(2), 2);
    double hf = (bits_min / double(U)) * std::log(2);
    uint64_t b = 2;
    while (b < uint64_t(bits_min)) b *= 2;
    *bits = b;
    *nh = int(std::ceil(hf));
    *nh_gate = int(uint64_t(hf));
}

// blocked layout: 512-bit blocks holding 256 positions of both filters
static uint64_t bloom_blocks(uint64_t bits) { return std::max<uint64_t>(1, bits / 256); }
static uint64_t bloom_words(const kc_ctx* c) {
    const uint64_t w = std::max<uint64_t>(1, (2 * c->bf_bits + 31) / 32);
    return c->bloom_blocked ? std::max<uint64_t>(w, 16 * bloom_blocks(c->bf_bits)) : w;
}

static int alloc_regions(kc_ctx* c);

// kc_route_table_device's buffers for n = parts x blocks entries (d_rhist moves: the level-3
// passes' pointer follows it and the kept counts are gone)
static int route_bufs(kc_ctx* c, uint64_t n) {
    if (n <= c->r_cap) return KC_OK;
    hipFree(c->d_rhist);
    hipFree(c->d_roff);
    hipFree(c->d_rbsum);
    c->d_rhist = nullptr;
    c->d_roff = c->d_rbsum = nullptr;
    c->r_cap = 0;
    c->own_valid = false;
    c->pb.own_hist = c->pbf.own_hist = nullptr;
    c->pb.own_parts = c->pbf.own_parts = 0;
    if (hipMalloc(&c->d_rhist, n * 4) != hipSuccess || hipMalloc(&c->d_roff, (n + 1) * 8) != hipSuccess ||
        hipMalloc(&c->d_rbsum, ((n + 4095) / 4096 + 2) * 8) != hipSuccess)
        return c->fail(KC_ERR_NOMEM, "route buffers allocation failed");
    c->r_cap = n;
    return KC_OK;
}

// Point the level-3 passes at d_rhist for the table's current geometry (kc_route_hint); the
// counts are valid again after a fresh level-3 pass (which writes every region)
static int own_prep(kc_ctx* c) {
    c->own_valid = false;
    c->pb.own_hist = c->pbf.own_hist = nullptr;
    c->pb.own_parts = c->pbf.own_parts = 0;
    if (!c->own_parts || !c->nbuckets) return KC_OK;
    const uint64_t nblk = (c->nbuckets + 255) / 256;  // = 2 R (BPR = 512)
    const int rc = route_bufs(c, c->own_parts * nblk);
    if (rc) return rc;
    c->pb.own_hist = c->pbf.own_hist = c->d_rhist;
    c->pb.own_parts = c->pbf.own_parts = c->own_parts;
    c->pb.own_nblk = c->pbf.own_nblk = nblk;
    return KC_OK;
}

// After a write into the table: the kept per-block counts stay valid through level-3 passes
// (k_p3 rewrites the counts of every region it writes; a fresh pass writes every region) and
// are lost by any other writer (direct atomics, the merge inserts)
static void own_after_write(kc_ctx* c, bool level3, bool fresh) {
    if (!level3) c->own_valid = false;
    else if (fresh) c->own_valid = c->pb.own_parts != 0;
}

// pow2_f1 != 0: R = F1 x F2 with F1 = pow2_f1 (the Bloom filter's coarse bins) and F2 a power
// of two, so the table's coarse bins are the filter's hash-prefix bins (level-1 reuse)
// phys_slots != 0: size the device table for that many k-mers instead of min_slots (the
// reference's capacity stays min_slots: kc_stats, KC_STRICT_CAPACITY)
static int alloc_table(kc_ctx* c, uint64_t min_slots, uint32_t pow2_f1 = 0, uint64_t phys_slots = 0) {
    c->min_slots = min_slots;
    // Kaarme's table holds exactly next_prime3mod4(min_slots) slots and dies when
    // full; open addressing on the GPU keeps 25 % headroom over that.  The table is
    // R = F1 * F2 regions of BPR 128-byte buckets (a region = one LDS-resident table).
    uint64_t want = std::max<uint64_t>(phys_slots ? phys_slots : min_slots, 64);
    want = want + want / 4;
    const uint64_t buckets = (want + c->S - 1) / c->S;
    const uint64_t regions = std::max<uint64_t>(1, (buckets + BPR - 1) / BPR);
    // R = F1 * F2 regions: F2 = 2^f2bits regions per level-1 bin, F1 ~ sqrt(R) <= 1024 bins
    // (multiply-shift region index, so R is not rounded up to a power of two)
    int rbits = 0;
    while ((1ULL << rbits) < regions) rbits++;
    if (pow2_f1) {
        int f1 = 0;
        while ((1u << f1) < pow2_f1) f1++;
        c->f2bits = std::max(0, rbits - f1);
        c->F2 = 1u << c->f2bits;
        c->F1 = pow2_f1;
        c->seg_ok = true;
    } else {
        // level 1 keeps F1 bins' arrays beside its tile in LDS (p1_lds_bytes), level 2 F2 bins'
        // (p2f_lds_bytes): big tables (C4, C5 shares) take more regions per coarse bin until
        // level 2 fits; for wide keys, if level 1 then does not fit, fewer, with level 2 at half
        // its workgroup (launch_p2f)
        auto f1_of = [&](int f2b) { return (uint32_t)((regions + (1ULL << f2b) - 1) >> f2b); };
        auto l2_fits = [&](int f2b, int nt) {
            const uint64_t b2 = std::max<uint64_t>(1, std::min<uint64_t>(64, 2048 / std::max<uint32_t>(1, f1_of(f2b))));
            return p2f_lds_bytes(c->W, 1u << f2b, (uint32_t)((2048 + b2 - 1) / b2), nt) <= LDS_BYTES;
        };
        auto l1_fits = [&](int f2b) { return p1_lds_bytes(c->W, f1_of(f2b)) <= LDS_BYTES; };
        int f1bits = std::min(10, (rbits + 1) / 2);
        while (f1bits < rbits && !l2_fits(rbits - f1bits, 0)) f1bits++;
        // level-1 runs of fewer than 8 keys per tile cost level 1 its second workgroup per CU
        // (launch_part_w): fewer, wider coarse bins while level 2 still fits (C4 share: 542 x 512
        // -> 271 x 1024 bins, k_p1 14.9 -> 9.9 ms, k_p2f 11.0 -> 12.3 ms, r03_ab_c4s_coarse_bins.txt)
        while (f1bits > 1 && (uint64_t)p1_tile(c->W) < 8ULL * f1_of(rbits - f1bits) &&
               l2_fits(rbits - f1bits + 1, 0))
            f1bits--;
        c->seg_ok = true;
        if (!l1_fits(rbits - f1bits)) {
            const int half = p2f_threads_w(c->W) / 2;
            f1bits = std::min(10, (rbits + 1) / 2);
            while (f1bits > 0 && !l1_fits(rbits - f1bits)) f1bits--;
            if (c->W <= 2 || !l1_fits(rbits - f1bits) || !l2_fits(rbits - f1bits, half)) {
                // beyond the segmented levels (wide keys in a multi-G-slot table, e.g. C5 on one
                // GPU): the exact layout, whose 256-thread levels hold smaller tiles
                const size_t tile = (size_t)COUNT_THREADS * run_width(c->W) * 8 * c->W + 16;
                auto fits_x = [&](uint64_t bins) { return bins * 32 + tile <= LDS_BYTES; };
                f1bits = 0;
                while (f1bits <= rbits && !(fits_x(f1_of(rbits - f1bits)) && fits_x(1ULL << (rbits - f1bits)))) f1bits++;
                if (f1bits > rbits) return c->fail(KC_ERR_ARG, "table too large for the partition levels");
                c->seg_ok = false;
            }
        }
        c->f2bits = rbits - f1bits;
        c->F2 = 1u << c->f2bits;
        c->F1 = f1_of(c->f2bits);
        // one-word keys: the level-2 records are 6 instead of 8 bytes once R >= 2^16
        // (kc_count_impl.h StoreRec6), so a table of 3/4 x 2^16 regions or more takes 2^16
        // (C2's -s 2e8: 61 184 -> 65 536 regions, 7 % more slots for 25 % fewer level-2 bytes)
        const uint64_t r0 = (uint64_t)c->F1 * c->F2;
        if (c->W == 1 && c->seg_ok && r0 >= 49152 && r0 < 65536 && l1_fits(c->f2bits)) {
            const uint32_t f1 = (uint32_t)((65536 + c->F2 - 1) / c->F2);
            if (p1_lds_bytes(1, f1) <= LDS_BYTES) c->F1 = f1;
        }
    }
    c->R = (uint64_t)c->F1 * c->F2;
    return alloc_regions(c);
}

// the table's memory for c->R regions (the geometry set by the caller)
static int alloc_regions(kc_ctx* c) {
    if (c->R >= (1ULL << 32)) return c->fail(KC_ERR_ARG, "table too large");  // 32-bit region index (kc_common.h)
    c->nbuckets = c->R * BPR;
    const size_t bytes = c->nbuckets * BUCKET_WORDS * sizeof(uint64_t);
    if (!c->d_table || bytes > c->table_cap_bytes) {  // else: reuse the previous allocation
        hipFree(c->d_table);
        c->d_table = nullptr;
        c->table_cap_bytes = 0;
        hipError_t e = hipMalloc(&c->d_table, bytes);
        if (e != hipSuccess)
            return c->fail(KC_ERR_NOMEM, "table allocation failed (" + std::to_string(bytes) + " bytes)");
        c->table_cap_bytes = bytes;
    }
    // zeroed lazily: a fresh partitioned pass writes every region from zero-filled LDS (C3's
    // counting pass: 0.66 ms of its 31 ms step was this memset), anything else that reads the
    // table first runs materialize_zero
    c->table_zero_pending = true;
    c->table_fresh = true;
    return own_prep(c);
}

static TableView table_view(const kc_ctx* c) {
    TableView tv;
    tv.buckets = c->d_table;
    tv.nbuckets = c->nbuckets;
    tv.R = c->R;
    tv.F1 = c->F1;
    tv.F2 = c->F2;
    tv.f2bits = c->f2bits;
    tv.W = c->W;
    tv.S = c->S;
    return tv;
}

// Perform a deferred table reset before the table is read or updated by anything but a
// fresh level-3 pass.
static int materialize_zero(kc_ctx* c, hipStream_t s) {
    if (!c->table_zero_pending || !c->d_table) return KC_OK;
    HIPCHK(c, hipMemsetAsync(c->d_table, 0, c->nbuckets * BUCKET_WORDS * sizeof(uint64_t), s));
    c->table_zero_pending = false;
    return KC_OK;
}

// Partition buffers for a batch of up to `syms` symbols (lazily grown).  seg: use the
// segmented single-pass layout (fixed-capacity segments, kc_count.hip OutSeg); its
// capacities are the expected fill of a segment (keys are hash-uniform over bins) plus
// 8 standard deviations plus 32, from the batch's symbol bound (>= its windows).  A
// batch whose keys still overflow a segment (e.g. one k-mer repeated millions of times
// inside one workgroup's range) is redone on the exact layout by the device itself.
// geometry of a partitioned pass: F1 coarse bins x F2 regions each (R regions), IW
// u64 words per item
struct PartGeo {
    uint32_t F1, F2;
    uint64_t R;
    int IW;
};
static PartGeo table_geo(const kc_ctx* c) { return PartGeo{c->F1, c->F2, c->R, c->W}; }

// The sizes of a partitioned pass over a batch of up to `syms` symbols (no allocation):
// level-1 workgroups, level-2 segments per bin, the segment capacities, the skew list and the key
// buffers' words.  slots > 1: the level-2 histogram and key buffers hold that many batches'
// segments (a deferred level 3, run_deferred), each record rec2 bytes (level2_record_bytes)
struct PartPlan {
    uint32_t nblk1, B2;
    uint64_t n1, n2, nbs;     // histogram entries: level 1, level 2, block sums
    uint64_t cap1, cap2;      // segment capacities (0: the exact layout)
    uint64_t spill_cap, spill_words, need1, need2;
};
static PartPlan part_plan(const kc_ctx* c, uint64_t syms, bool seg, const PartGeo& g, uint32_t bins1, uint32_t slots,
                          uint64_t rec2 = 0, bool tight = false) {
    PartPlan p{};
    const uint64_t tile = (uint64_t)COUNT_THREADS * run_width(c->W);
    p.nblk1 = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(2048, (syms + tile - 1) / tile));
    p.B2 = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(64, 2048 / g.F1));
    // every array is sized for the geometry of THIS call (a Bloom job re-sizes the table
    // after each Bloom pass, so F1 and R may grow between calls on one context)
    p.n1 = (uint64_t)std::max<uint32_t>(g.F1, bins1) * 2048;  // level-1 bins x max workgroups
    p.n2 = g.R * p.B2 * slots;
    p.nbs = (std::max(p.n1, p.n2) + 4095) / 4096 + 2;
    if (seg) {
        // tight (a deferred pass): e + 3.5 sigma + 8.  Its keys past a segment's end (a few segments
        // in 10^4 overflow, by a few keys) join the group's skew list, which is inserted once after
        // the group's level 3 (run_deferred), so the slots of more batches fit beside the table (C5
        // on one GPU: 54.2 -> 43.4 GB per batch, groups of 2 -> 3).  (At 3 sigma, C5's ~54 K spilled
        // keys per batch touched ~100 K regions per group in the list's level 3: 12 ms per job.)
        const double sd = tight ? 3.5 : 8.0, add = tight ? 8.0 : 32.0;
        auto capacity = [&](double e) { return ((uint64_t)std::ceil(e + sd * std::sqrt(e) + add) + 7) / 8 * 8; };
        const uint64_t t1 = (uint64_t)p1_tile_max(c->W);  // k_p1<..., OutSeg> rounds block ranges to its tile
        const uint64_t per1 = ((syms + p.nblk1 - 1) / p.nblk1 + t1 - 1) / t1 * t1;  // symbols per level-1 block
        const uint64_t nseg = (p.nblk1 + p.B2 - 1) / p.B2;                           // level-1 segments per p2 block
        const double d = c->win_density;  // windows per symbol (1 for tokenized input)
        p.cap1 = capacity((double)per1 * d / g.F1);
        p.cap2 = capacity((double)nseg * per1 * d / g.F1 / g.F2);
        if (const char* v = std::getenv("KC_SEG_CAP")) p.cap1 = p.cap2 = std::max<uint64_t>(1, std::strtoull(v, 0, 10));
        // the segment walks index a virtual run with 32-bit offsets
        if (nseg * p.cap1 >= (1ULL << 31) || (uint64_t)p.B2 * p.cap2 * slots >= (1ULL << 31)) p.cap1 = p.cap2 = 0;
    }
    // the skew list of a segmented batch: {key words, count} records of keys past a segment's
    // end and of repeated windows (Bloom pass: plain keys), an eighth of the windows before the
    // batch falls back to the exact layout; its exact pipeline runs through the key buffers
    const uint64_t wins = c->win_density < 1.0 ? (uint64_t)((double)syms * c->win_density) + 1024 : syms;
    if (p.cap1) {
        // (a deferred pass's list takes its group's few spilled keys: a sixteenth)
        p.spill_cap = std::max<uint64_t>(1 << 16, wins / (tight ? 16 : 8));
        if (const char* v = std::getenv("KC_SPILL_CAP")) p.spill_cap = std::strtoull(v, 0, 10);  // tests
    }
    p.spill_words = p.spill_cap * (g.IW + 1);
    p.need1 = std::max(std::max<uint64_t>(wins, (uint64_t)g.F1 * p.nblk1 * p.cap1) * g.IW, p.spill_words);
    // one batch's level 2 in W-word items; a deferred group's slots in level-2 records (the exact
    // pipeline of a batch's tail, which writes W-word items, runs after its group's level 3)
    const uint64_t l2 = slots > 1 && rec2 ? (g.R * p.B2 * p.cap2 * slots * rec2 + 7) / 8 : g.R * p.B2 * p.cap2 * g.IW;
    p.need2 = std::max(std::max<uint64_t>(wins * g.IW, l2), p.spill_words);
    // (the levels' record loads are 12 or 16 bytes wide whatever the record: a last 8- or
    // 12-byte record's load reads past it)
    p.need1 += 2;
    p.need2 += 2;
    return p;
}

// Partition buffers for a batch of up to `syms` symbols (lazily grown): part_plan's sizes
static int ensure_part_geo(kc_ctx* c, uint64_t syms, bool seg, const PartGeo& g, PartBufs& pb, PartCap& cap,
                           uint32_t bins1 = 0, uint32_t slots = 1, uint64_t rec2 = 0) {
    const PartPlan p = part_plan(c, syms, seg, g, bins1, slots, rec2, slots > 1);
    const uint64_t n1 = p.n1, n2 = p.n2, nbs = p.nbs;
    if (n1 > cap.h1) {
        hipFree(pb.hist1);
        hipFree(pb.off1);
        pb.hist1 = nullptr;
        pb.off1 = nullptr;
        cap.h1 = 0;
        if (hipMalloc(&pb.hist1, n1 * 4) != hipSuccess || hipMalloc(&pb.off1, (n1 + 1) * 8) != hipSuccess)
            return c->fail(KC_ERR_NOMEM, "partition histogram allocation failed");
        cap.h1 = n1;
    }
    if (n2 > cap.h2) {
        hipFree(pb.hist2);
        hipFree(pb.off2);
        pb.hist2 = nullptr;
        pb.off2 = nullptr;
        cap.h2 = 0;
        if (hipMalloc(&pb.hist2, n2 * 4) != hipSuccess || hipMalloc(&pb.off2, (n2 + 1) * 8) != hipSuccess)
            return c->fail(KC_ERR_NOMEM, "partition histogram allocation failed");
        cap.h2 = n2;
    }
    if (nbs > cap.bs) {
        hipFree(pb.bsum);
        pb.bsum = nullptr;
        cap.bs = 0;
        if (hipMalloc(&pb.bsum, nbs * 8) != hipSuccess)
            return c->fail(KC_ERR_NOMEM, "partition histogram allocation failed");
        cap.bs = nbs;
    }
    const uint64_t cap1 = p.cap1, cap2 = p.cap2, spill_cap = p.spill_cap, spill_words = p.spill_words;
    const uint64_t need1 = p.need1, need2 = p.need2;
    const uint32_t nblk1 = p.nblk1, B2 = p.B2;
    auto grow = [&](uint64_t** buf, uint64_t* have, uint64_t need) -> int {
        if (need <= *have) return KC_OK;
        hipFree(*buf);
        *buf = nullptr;
        *have = 0;
        const size_t bytes = (size_t)need * 8;
        if (hipMalloc(buf, bytes) != hipSuccess)
            return c->fail(KC_ERR_NOMEM, "partition key buffer allocation failed (" + std::to_string(bytes) + " bytes)");
        *have = need;
        return KC_OK;
    };
    int rc = grow(&c->d_keys1, &c->k1_words, need1);
    if (rc) return rc;
    rc = grow(&c->d_keys2, &c->k2_words, need2);
    if (rc) return rc;
    if (spill_cap && (rc = grow(&c->d_spill, &c->spill_words, spill_words))) return rc;
    pb.spill = c->d_spill;
    pb.spill_cap = spill_cap;
    pb.keys1 = c->d_keys1;
    pb.keys2 = c->d_keys2;
    pb.nblk1 = nblk1;
    pb.B2 = B2;
    pb.cap1 = cap1;
    pb.cap2 = cap2;
    return KC_OK;
}
// the table's levels
static int ensure_part(kc_ctx* c, uint64_t syms, bool seg, uint32_t bins1 = 0, uint32_t slots = 1) {
    seg = seg && c->seg_ok;
    return ensure_part_geo(c, syms, seg, table_geo(c), c->pb, c->pb_cap, bins1, slots,
                           slots > 1 ? level2_record_bytes(c->W, c->cfg.k, c->R) : 0);
}

// KC_INSERT_PATH (tests, include/kc_api.h knobs): direct | partitioned | exact forces one insert
// path for every batch; unset = chosen per batch by the cost rules below
enum class PathKnob { Auto, Direct, Partitioned, Exact };
static PathKnob insert_path_knob() {
    const char* v = std::getenv("KC_INSERT_PATH");
    if (!v) return PathKnob::Auto;
    if (!std::strcmp(v, "direct")) return PathKnob::Direct;
    if (!std::strcmp(v, "partitioned")) return PathKnob::Partitioned;
    if (!std::strcmp(v, "exact")) return PathKnob::Exact;
    return PathKnob::Auto;
}
// KC_DEBUG=1: the host's decisions (partition reuse, deferred level 3) on stderr
static bool debug_on() {
    const char* v = std::getenv("KC_DEBUG");
    return v && *v && *v != '0';
}

// Insert path per batch: the partitioned pipeline moves ~(4W+1)*8 bytes per window
// plus two sweeps of the table; the direct path is bound by scattered device atomics
// (~20 G/s on MI355X, i.e. ~275 bytes-equivalent per window at ~5.5 TB/s).
static bool use_partitioned(const kc_ctx* c, uint64_t syms) {
    const PathKnob p = insert_path_knob();
    if (p != PathKnob::Auto) return p != PathKnob::Direct;
    const double table_bytes = (double)c->nbuckets * 128.0;
    return (double)syms * 275.0 > (double)syms * (4.0 * c->W + 1) * 8.0 + 2.0 * table_bytes;
}

// Bloom pass 1 (blocked layout): the partitioned pass moves one u64 per window three
// times plus two sweeps of the filter; the direct pass costs a scattered 64-byte line
// RMW with up to ceil(hf) device-scope atomics per window.
static bool use_partitioned_bloom(const kc_ctx* c, uint64_t syms) {
    const PathKnob p = insert_path_knob();
    if (p != PathKnob::Auto) return p != PathKnob::Direct;
    const double filter_bytes = (double)bloom_words(c) * 4.0;
    return (double)syms * 275.0 > (double)syms * 5.0 * 8.0 + 2.0 * filter_bytes;
}

// The device entry points run on the caller's stream, ordered after the work already
// enqueued there (NULL = the HIP null stream, PyTorch's default current stream), and
// hand over to/from the context's own stream with events.
static hipStream_t pick_stream(kc_ctx* c, void* s) {
    (void)c;
    return (hipStream_t)s;
}

// ------------------------------------------------------------------------------
// batch execution
// ------------------------------------------------------------------------------
// src: the bytes the chunk descriptors' src_off point into (the host stage, or a
// device-resident image read in place)
// The tail of a segmented batch (the skew list, the batch's bookkeeping, the exact pipeline
// behind the device overflow gate) does nothing unless the single-pass levels left a skew list
// or overflowed.  For device images the host reads those two counters after the main phase
// (the call waits for its batch) and launches the tail only when needed: ~20 idle kernel
// launches and two region-grid passes less per batch (0.25 ms of C2's 15.9 ms step).  Images
// of several batches and host chunks keep the device gate (their batches queue behind each
// other).
static int tail_needed(kc_ctx* c, hipStream_t s, bool* need) {
    unsigned long long f[2] = {0, 0};
    HIPCHK(c, hipMemcpyAsync(&f[0], &c->d_ctr->part_overflow, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(&f[1], &c->d_ctr->spill_n, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    *need = f[0] != 0 || f[1] != 0;
    return KC_OK;
}

// a device counter set from the host, in stream order
static hipError_t set_dev_u64(unsigned long long* p, uint64_t v, hipStream_t s) {
    hipError_t e = hipMemsetD32Async((hipDeviceptr_t)p, (int)(uint32_t)v, 1, s);
    if (e == hipSuccess) e = hipMemsetD32Async((hipDeviceptr_t)((uint32_t*)p + 1), (int)(uint32_t)(v >> 32), 1, s);
    return e;
}

// The level-3 pass of the deferred group (run_deferred): the waiting batches' segments, slots of
// batches that did not fill the group zeroed first (their fills are a previous group's)
static int flush_deferred(kc_ctx* c, const PackedView& sv, uint64_t syms, int mode, const TableView& tv,
                          const BloomView& bv, PartBufs pb, hipStream_t s, bool overflowed) {
    const uint32_t G = c->defer_g, B2 = c->pb.B2;
    // (the batch that overflowed: its segments are not all written; its tail redoes it)
    const uint32_t keep = overflowed ? c->defer_n - 1 : c->defer_n;
    if (keep < G)
        HIPCHK(c, hipMemset2DAsync(c->pb.hist2 + (uint64_t)keep * B2, (size_t)G * B2 * 4, 0, (size_t)(G - keep) * B2 * 4,
                                   c->R, s));
    if (overflowed) HIPCHK(c, launch_hold_overflow(c->d_ctr, 0, s));
    HIPCHK(c, launch_count_partitioned(sv, syms, c->cfg.k, mode, tv, bv, c->d_ctr, pb, c->table_fresh, s, PH_L3));
    if (overflowed) HIPCHK(c, launch_hold_overflow(c->d_ctr, 1, s));
    c->table_zero_pending = false;  // a fresh level 3 writes every region
    own_after_write(c, true, c->table_fresh);
    c->table_fresh = false;
    c->defer_n = 0;
    c->defer_groups++;
    return KC_OK;
}

// One batch of a deferred counting pass: levels 1-2 into the batch's slot of the group's level-2
// segments; the group's level 3 when the group is full, at the pass's last batch, or when this
// batch needs its tail (a skew list, or segments that overflowed: the tail's exact pipeline uses
// the key buffers as scratch, so the waiting segments are inserted first).  The host reads the
// batch's two flags (it waits for the batch) before queueing the next one.
static int run_deferred(kc_ctx* c, const PackedView& sv, uint64_t syms, int mode, const TableView& tv,
                        const BloomView& bv, hipStream_t s) {
    PartBufs pb = c->pb;
    pb.b2t = c->defer_g * pb.B2;
    pb.b2off = c->defer_n * pb.B2;
    pb.keep_skew = c->defer_n > 0;  // (the group's skew list so far stays)
    HIPCHK(c, launch_count_partitioned(sv, syms, c->cfg.k, mode, tv, bv, c->d_ctr, pb, c->table_fresh, s, PH_L12));
    c->defer_n++;
    unsigned long long f[3] = {0, 0, 0};
    HIPCHK(c, hipMemcpyAsync(&f[0], &c->d_ctr->part_overflow, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(&f[1], &c->d_ctr->spill_n, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(&f[2], &c->d_ctr->heavy_n, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    const bool overflowed = f[0] != 0;
    // a skew list alone does not end the group: the next batch appends to it
    if (!overflowed && c->defer_n < c->defer_g && !c->defer_last) {
        c->skew_prev = f[1];
        c->heavy_prev = f[2];
        return KC_OK;
    }
    int rc = flush_deferred(c, sv, syms, mode, tv, bv, pb, s, overflowed);
    if (rc) return rc;
    if (overflowed && c->skew_prev) {
        // this batch is redone by the exact pipeline (its tail); the list's first skew_prev entries
        // are the group's earlier batches' and are inserted first, with the overflow flag held
        HIPCHK(c, launch_hold_overflow(c->d_ctr, 0, s));
        HIPCHK(c, set_dev_u64(&c->d_ctr->spill_n, c->skew_prev, s));
        HIPCHK(c, set_dev_u64(&c->d_ctr->heavy_n, c->heavy_prev, s));
        HIPCHK(c, launch_count_partitioned(sv, syms, c->cfg.k, mode, tv, bv, c->d_ctr, c->pb, c->table_fresh, s,
                                           PH_TAIL));
        HIPCHK(c, set_dev_u64(&c->d_ctr->spill_n, 0, s));
        HIPCHK(c, set_dev_u64(&c->d_ctr->heavy_n, 0, s));
        HIPCHK(c, launch_hold_overflow(c->d_ctr, 1, s));
    }
    c->skew_prev = c->heavy_prev = 0;
    if (overflowed || f[1] != 0)
        HIPCHK(c, launch_count_partitioned(sv, syms, c->cfg.k, mode, tv, bv, c->d_ctr, c->pb, c->table_fresh, s,
                                           PH_TAIL));
    return KC_OK;
}

// pre: a symbol stream already in HBM (a received super-k-mer stream, kc_count_packed_device) of
// `used` symbols instead of chunks to tokenize (src, nchunks and fmt unused); pre_len: the device
// word holding its actual length when `used` only bounds it (a batch the estimate pass tokenized)
static int run_batch(kc_ctx* c, const uint8_t* src, uint64_t used, uint64_t nchunks, int fmt, int pass, hipStream_t s,
                     hipEvent_t ev_start = nullptr, hipEvent_t ev_gather = nullptr, bool keep = false,
                     bool host_gate = false, const PackedView* pre = nullptr, const uint64_t* pre_len = nullptr) {
    const uint64_t ntiles = used / TILE;
    if (!pre && ntiles == 0) return KC_OK;
    if (pre && used == 0) return KC_OK;
    if (pass == 3) {  // the distinct-count sketch (kc_estimate_distinct_device): tokenize + k_hll
        PackedView v{c->d_pk, c->d_bk};
        const uint64_t words = (used + nchunks) / 32 + 4;
        const bool kept = c->keep_target && c->keep_woff + words <= c->keep_cap && c->kept.size() < c->kept_len_cap;
        if (kept) {  // (kept for the counting pass)
            v = PackedView{c->keep_pk + c->keep_woff, c->keep_bk + c->keep_woff};
            c->kept.emplace_back(c->keep_woff, used + nchunks);
            c->keep_woff += words;
        } else {
            c->keep_target = false;
        }
        HIPCHK(c, launch_tokenize(src, ntiles, c->d_chunks, (int)nchunks, fmt, c->d_tiles, c->d_touts, c->d_tblk, v,
                                  used + nchunks, c->d_ctr, s));
        if (kept)  // the batch's stream length (the tokenizer's, below the bound)
            HIPCHK(c, hipMemcpyAsync(c->d_kept_len + c->kept.size() - 1, &c->d_ctr->stream_len, 8,
                                     hipMemcpyDeviceToDevice, s));
        HIPCHK(c, launch_hll(v, c->cfg.k, c->W, c->d_ctr, c->d_hll, s));
        if (kept)  // the windows so far (the batch's: the difference to the previous batch's)
            HIPCHK(c, hipMemcpyAsync(c->d_kept_win + c->kept.size() - 1, &c->d_ctr->est_windows, 8,
                                     hipMemcpyDeviceToDevice, s));
        return KC_OK;
    }
    if (pass == 4) {  // super-k-mer routing (kc_route_superkmers_device): tokenize + k_skm_route
        const PackedView v{c->d_pk, c->d_bk};
        HIPCHK(c, launch_tokenize(src, ntiles, c->d_chunks, (int)nchunks, fmt, c->d_tiles, c->d_touts, c->d_tblk, v,
                                  used + nchunks, c->d_ctr, s));
        HIPCHK(c, launch_skm_route(v, c->d_ctr, used + nchunks, c->cfg.k, c->skm_m, c->skm_shards, c->skm_pk,
                                   c->skm_bk, c->skm_cap, c->d_skm, c->d_skm + SKM_MAX_SHARDS,
                                   c->d_skm + 2 * SKM_MAX_SHARDS, s));
        return KC_OK;
    }
    std::array<hipEvent_t, 4> ev{ev_start, ev_gather, nullptr, nullptr};
    if (c->profiling) {
        if (!ev[0]) {
            ev[0] = c->get_event();
            ev[1] = c->get_event();
            HIPCHK(c, hipEventRecord(ev[0], s));
            HIPCHK(c, hipEventRecord(ev[1], s));
        }
        ev[2] = c->get_event();
        ev[3] = c->get_event();
    }
    const PackedView sv = pre ? *pre : PackedView{c->d_pk, c->d_bk};
    if (pre) {  // (the stream's length where the tokenizer would have left it)
        if (pre_len) {
            HIPCHK(c, hipMemcpyAsync(&c->d_ctr->stream_len, pre_len, 8, hipMemcpyDeviceToDevice, s));
        } else {
            HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)&c->d_ctr->stream_len, (int)(uint32_t)used, 1, s));
            HIPCHK(c, hipMemsetD32Async((hipDeviceptr_t)((uint32_t*)&c->d_ctr->stream_len + 1),
                                        (int)(uint32_t)(used >> 32), 1, s));
        }
        nchunks = 0;
    } else {
        HIPCHK(c, launch_tokenize(src, ntiles, c->d_chunks, (int)nchunks, fmt, c->d_tiles, c->d_touts, c->d_tblk, sv,
                                  used + nchunks, c->d_ctr, s));
    }
    if (c->profiling) HIPCHK(c, hipEventRecord(ev[2], s));
    TableView tv = table_view(c);
    BloomView bv{c->d_bloom, c->bf_bits ? c->bf_bits - 1 : 0, c->nh, c->nh_gate, c->bloom_blocked,
                 bloom_blocks(c->bf_bits)};
    int mode;
    if (pass == 1) mode = 1;
    else mode = (c->cfg.bf_enable && c->cfg.mode != 1) ? 2 : 0;  // -m 1 -b ignores the filter (main.cpp:482-489)
    const uint64_t syms = used + nchunks;
    if (mode == 1) {
        c->bloom_batches++;
        c->reuse_kept = false;
    }
    if (mode == 1 && c->bloom_blocked && use_partitioned_bloom(c, syms)) {
        const bool seg = insert_path_knob() != PathKnob::Exact;
        keep = keep && seg;  // (the exact layout does not keep: its level 1 moves word 0 only)
        keep = keep && c->fgeo.R != 0;
        const PartGeo g = keep ? PartGeo{c->fgeo.F1, c->fgeo.F2, c->fgeo.R, c->W}
                               : PartGeo{c->bgeo.F1, c->bgeo.F2, c->bgeo.R, 1};
        int rc = ensure_part_geo(c, syms, seg, g, c->pbf, c->pbf_cap);
        if (rc) return rc;
        c->pbf.keep_fill = c->pbf.keep_fill2 = nullptr;
        if (keep) {  // copies of the kept partitions' segment fills
            auto grow = [&](uint32_t** p, uint64_t* cap, uint64_t n) -> int {
                if (n <= *cap) return KC_OK;
                hipFree(*p);
                *p = nullptr;
                *cap = 0;
                if (hipMalloc(p, n * 4) != hipSuccess) return c->fail(KC_ERR_NOMEM, "partition fill copy allocation failed");
                *cap = n;
                return KC_OK;
            };
            if ((rc = grow(&c->d_keep_fill, &c->keep_fill_cap, (uint64_t)c->fgeo.F1 * c->pbf.nblk1)) ||
                (rc = grow(&c->d_keep_fill2, &c->keep_fill2_cap, c->fgeo.R * c->pbf.B2)))
                return rc;
            c->pbf.keep_fill = c->d_keep_fill;
            c->pbf.keep_fill2 = c->d_keep_fill2;
        }
        // two-word keys: the kept levels as 12-byte records (kc_count_impl.h Rec12) when a record
        // holds the table key's bits below its bin: hb + 1 + xb <= 32 at both levels
        c->pbf.rec12 = 0;
        if (keep && c->W == 2) {
            int f1 = 0, rb = 0;
            while ((1u << f1) < c->fgeo.F1) f1++;
            while ((1ULL << rb) < c->fgeo.R) rb++;
            const int hb = std::max(0, 2 * c->cfg.k - 96);
            int b2s = 0;
            while ((1u << b2s) < c->pbf.B2) b2s++;
            if (hb + 1 + (32 - f1) <= 32 && hb + 1 + (32 - rb) <= 32 && f1 >= 1 && (1u << b2s) == c->pbf.B2) {
                c->pbf.rec12 = R12_P1 | R12_IN | R12_OUT | R12_L2;
                c->pbf.r12_hb = hb;
                c->pbf.r12_xb1 = 32 - f1;
                c->pbf.r12_xb2 = 32 - rb;
                c->pbf.r12_b2s = b2s;
            }
        }
        const bool split = host_gate && c->pbf.cap1 != 0;
        bool tail = false;
        HIPCHK(c, launch_bloom_partitioned(sv, c->cfg.k, c->W, bv, c->bgeo, c->fgeo, c->d_ctr, c->pbf, c->bloom_fresh,
                                           keep ? 1 : 0, s, split ? PH_MAIN : PH_ALL));
        if (split && (rc = tail_needed(c, s, &tail))) return rc;
        if (tail)
            HIPCHK(c, launch_bloom_partitioned(sv, c->cfg.k, c->W, bv, c->bgeo, c->fgeo, c->d_ctr, c->pbf,
                                               c->bloom_fresh, keep ? 1 : 0, s, PH_TAIL));
        c->bloom_fresh = false;
        c->reuse_kept = keep;
    } else if (mode != 1 && c->defer_on) {  // (device_pass chose the partitioned segmented path)
        int rc = ensure_part(c, std::max(syms, c->defer_syms), true, 0, c->defer_g);
        if (rc) return rc;
        if (c->pb.cap1 == 0) return c->fail(KC_ERR_STATE, "deferred level 3 without segmented levels");
        if ((rc = run_deferred(c, sv, syms, mode, tv, bv, s))) return rc;
    } else if (mode != 1 && use_partitioned(c, syms)) {
        int rc = ensure_part(c, syms, insert_path_knob() != PathKnob::Exact);
        if (rc) return rc;
        const bool split = host_gate && c->pb.cap1 != 0;
        HIPCHK(c, launch_count_partitioned(sv, syms, c->cfg.k, mode, tv, bv, c->d_ctr, c->pb, c->table_fresh, s,
                                           split ? PH_MAIN : PH_ALL));
        bool tail = false;
        if (split && (rc = tail_needed(c, s, &tail))) return rc;
        if (tail)
            HIPCHK(c, launch_count_partitioned(sv, syms, c->cfg.k, mode, tv, bv, c->d_ctr, c->pb, c->table_fresh, s,
                                               PH_TAIL));
        c->table_zero_pending = false;  // the fresh pass wrote every region
        own_after_write(c, true, c->table_fresh);
    } else {
        if (mode != 1) {
            const int rc = materialize_zero(c, s);
            if (rc) return rc;
            own_after_write(c, false, false);
        }
        HIPCHK(c, launch_count(sv, syms, c->cfg.k, mode, tv, bv, c->d_ctr, s));
        if (mode == 1) c->bloom_fresh = false;
    }
    if (mode != 1 && !c->defer_on) c->table_fresh = false;  // (a deferred pass: its level 3 clears it)
    if (c->profiling) {
        HIPCHK(c, hipEventRecord(ev[3], s));
        c->ev_pending.push_back(ev);
        c->pending_symbols_bound.push_back(used + nchunks);
    }
    return KC_OK;
}

static int flush_host(kc_ctx* c) {
    if (c->cur_n == 0) return KC_OK;
    const int b = c->cur;
    HIPCHK(c, hipMemcpyAsync(c->d_stage, c->h_stage[b], c->cur_used, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->d_chunks, c->h_desc[b], c->cur_n * sizeof(ChunkDesc), hipMemcpyHostToDevice,
                             c->stream));
    HIPCHK(c, hipEventRecord(c->h_free[b], c->stream));
    int rc = run_batch(c, c->d_stage, c->cur_used, c->cur_n, c->cur_fmt, c->cur_pass, c->stream);
    if (rc) return rc;
    c->cur ^= 1;
    c->cur_used = 0;
    c->cur_n = 0;
    HIPCHK(c, hipEventSynchronize(c->h_free[c->cur]));  // buffer we fill next is no longer read
    return KC_OK;
}

static int add_host_chunk(kc_ctx* c, const uint8_t* buf, size_t len, int fmt, int bh, int pass) {
    if (!buf && len) return c->fail(KC_ERR_ARG, "null buffer");
    if (fmt != KC_FMT_FASTA && fmt != KC_FMT_FASTQ && fmt != KC_FMT_PLAIN) return c->fail(KC_ERR_ARG, "unknown format");
    if (len == 0) return KC_OK;
    const uint64_t need = round_up(len, TILE);
    if (need > c->batch_bytes) return c->fail(KC_ERR_ARG, "chunk larger than the staging batch");
    if (c->cur_n && (c->cur_fmt != fmt || c->cur_pass != pass || c->cur_used + need > c->batch_bytes ||
                     c->cur_n + 1 > c->max_chunks)) {
        int rc = flush_host(c);
        if (rc) return rc;
    }
    ChunkDesc d;
    d.src_off = c->cur_used;  // host chunks are tokenized from the stage itself
    d.stage_off = c->cur_used;
    d.len = len;
    d.bh = bh ? 1 : 0;
    d.pad = 0;
    if (!c->h_stage[c->cur]) {  // host chunks: two pinned stages + the device stage, on first use
        for (int i = 0; i < 2; i++)
            if (!c->h_stage[i] && hipHostMalloc(&c->h_stage[i], c->batch_bytes, hipHostMallocDefault) != hipSuccess)
                return c->fail(KC_ERR_NOMEM, "pinned staging allocation failed");
        if (!c->d_stage && hipMalloc(&c->d_stage, c->batch_bytes) != hipSuccess)
            return c->fail(KC_ERR_NOMEM, "device stage allocation failed");
    }
    std::memcpy(c->h_stage[c->cur] + c->cur_used, buf, len);
    c->h_desc[c->cur][c->cur_n++] = d;
    c->cur_used += need;
    c->cur_fmt = fmt;
    c->cur_pass = pass;
    if (pass == 0) { c->n_chunks++; c->n_bytes += len; }
    return KC_OK;
}

static bool reuse_enabled() {
    const char* v = std::getenv("KC_REUSE");
    return !(v && *v == '0');
}

// The counting pass from the Bloom pass's kept level-1 output (see kc_ctx, level-1 reuse).
// Sets *done when the pass ran; otherwise (different input, changed bytes, overflow) the
// caller runs the ordinary pass and nothing was counted.
static int count_reused(kc_ctx* c, const uint8_t* img, const kc_chunk* chunks, size_t n, int fmt, hipStream_t s,
                        bool* done) {
    *done = false;
    if (img != c->reuse_img || fmt != c->reuse_fmt) {
        if (debug_on()) std::fprintf(stderr, "reuse: another image or format\n");
        return KC_OK;
    }
    std::vector<ChunkDesc> b;
    uint64_t used = 0, max_len = 0, bytes = 0;
    for (size_t i = 0; i < n; i++) {
        if (chunks[i].len == 0) continue;
        ChunkDesc d;
        d.src_off = chunks[i].off;
        d.stage_off = used;
        d.len = chunks[i].len;
        d.bh = chunks[i].broken_header ? 1 : 0;
        d.pad = 0;
        b.push_back(d);
        used += round_up(chunks[i].len, TILE);
        max_len = std::max<uint64_t>(max_len, d.len);
        bytes += d.len;
    }
    if (b.size() != c->reuse_chunks.size() || used != c->reuse_used) return KC_OK;
    for (size_t i = 0; i < b.size(); i++) {
        const ChunkDesc &x = b[i], &y = c->reuse_chunks[i];
        if (x.src_off != y.src_off || x.len != y.len || x.bh != y.bh) return KC_OK;
    }
    int rc = flush_host(c);  // keep order with staged host chunks
    if (rc) return rc;
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->xev, 0));
    }
    std::array<hipEvent_t, 4> ev{nullptr, nullptr, nullptr, nullptr};
    if (c->profiling)
        for (auto& e : ev) e = c->get_event();
    auto release = [&]() {
        for (auto e : ev)
            if (e) c->ev_pool.push_back(e);
    };
    if (ev[0]) {
        HIPCHK(c, hipEventRecord(ev[0], s));
        HIPCHK(c, hipEventRecord(ev[1], s));
    }
    // the bytes must be the Bloom pass's: same checksum.  It runs on the aux stream beside the
    // counting pass from the partitions (which reads no input byte); a mismatch restores the
    // counters and drops the table before the ordinary pass (C3: 0.35 ms off the step)
    std::memcpy(c->h_desc[c->cur], b.data(), b.size() * sizeof(ChunkDesc));
    HIPCHK(c, hipMemcpyAsync(c->d_chunks, c->h_desc[c->cur], b.size() * sizeof(ChunkDesc), hipMemcpyHostToDevice, s));
    if (!c->aux) {
        HIPCHK(c, hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
        for (auto& e : c->aev) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    HIPCHK(c, hipEventRecord(c->aev[0], s));
    HIPCHK(c, hipStreamWaitEvent(c->aux, c->aev[0], 0));
    HIPCHK(c, launch_checksum(img, c->d_chunks, (int)b.size(), max_len, c->d_sum, c->aux));
    HIPCHK(c, hipMemcpyAsync(c->h_part, c->d_sum, sizeof(c->h_part), hipMemcpyDeviceToHost, c->aux));
    HIPCHK(c, hipEventRecord(c->aev[1], c->aux));
    auto same_bytes = [&](bool* same) -> int {  // waits for the checksum
        HIPCHK(c, hipEventSynchronize(c->aev[1]));
        unsigned long long sum = 0;
        for (auto v : c->h_part) sum += v;
        *same = sum == c->reuse_sum;
        if (!*same && debug_on()) std::fprintf(stderr, "reuse: checksum differs\n");
        return KC_OK;
    };
    if (ev[2]) HIPCHK(c, hipEventRecord(ev[2], s));
    bool same = false;
    const uint64_t syms = used + b.size();
    // the table's partition buffers for this batch, with the Bloom pass's partitions as its
    // level 1 (and level 2); the kept buffers must not have moved
    if ((rc = ensure_part(c, syms, true))) return rc;
    PartBufs pr = c->pb;
    if (pr.keys1 != c->pbf.keys1 || (c->reuse_level == 2 && pr.keys2 != c->pbf.keys2) || pr.nblk1 != c->pbf.nblk1 ||
        pr.B2 != c->pbf.B2 || pr.cap1 != c->pbf.cap1 || pr.cap1 == 0 || c->F1 != c->fgeo.F1) {
        if (debug_on()) std::fprintf(stderr, "reuse: partition geometry differs\n");
        HIPCHK(c, hipEventSynchronize(c->aev[1]));
        release();
        return KC_OK;
    }
    pr.hist1 = c->d_keep_fill;
    // the kept records' format: level 2 read by level 3, or level 1 read by level 2 (which then
    // writes whole keys in the table's own geometry)
    pr.rec12 = c->pbf.rec12 ? (c->reuse_level == 2 ? R12_L2 : R12_IN) : 0;
    pr.r12_hb = c->pbf.r12_hb;
    pr.r12_xb1 = c->pbf.r12_xb1;
    pr.r12_xb2 = c->pbf.r12_xb2;
    pr.r12_b2s = c->pbf.r12_b2s;
    if (c->reuse_level == 2) {  // a table region = fgeo.R / R consecutive fine bins
        pr.hist2 = c->d_keep_fill2;
        pr.cap2 = c->pbf.cap2;
        pr.B2 = (uint32_t)(c->fgeo.R / c->R) * c->pbf.B2;
    }
    const BloomView bv{c->d_bloom, c->bf_bits ? c->bf_bits - 1 : 0, c->nh, c->nh_gate, c->bloom_blocked,
                       bloom_blocks(c->bf_bits)};
    // the counters as they were, for a redo (other bytes, or a table region that overflowed)
    DevCounters before;
    HIPCHK(c, hipMemcpyAsync(&before, c->d_ctr, sizeof(before), hipMemcpyDeviceToHost, s));
    // -m 1 -b counts every window (the reference ignores its filter, main.cpp:482-489)
    HIPCHK(c, launch_count_reuse(c->W, table_view(c), bv, c->d_ctr, pr, c->table_fresh, c->reuse_level,
                                 c->cfg.mode != 1, c->reuse_windows, s));
    if (ev[3]) HIPCHK(c, hipEventRecord(ev[3], s));
    unsigned long long ovf = 0, full = 0;
    HIPCHK(c, hipMemcpyAsync(&ovf, &c->d_ctr->part_overflow, sizeof(ovf), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipMemcpyAsync(&full, &c->d_ctr->overflow, sizeof(full), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if ((rc = same_bytes(&same))) return rc;
    if (!same || ovf || full != before.overflow) {
        // other bytes than the Bloom pass's, a full skew list, or a region of the table sized for
        // the gated k-mers that overflowed: the ordinary counting pass redoes the batch into a
        // fresh reference-sized table (2 * new_in_second), with the counters as they were
        if (debug_on() && same)
            std::fprintf(stderr, "reuse: %s, redo\n", ovf ? "level 2 overflowed" : "table region overflowed");
        HIPCHK(c, hipMemcpyAsync(c->d_ctr, &before, sizeof(before), hipMemcpyHostToDevice, s));
        HIPCHK(c, hipStreamSynchronize(s));
        release();
        return alloc_table(c, c->min_slots);
    }
    own_after_write(c, true, c->table_fresh);
    c->table_fresh = false;
    c->table_zero_pending = false;  // the fresh level 3 wrote every region
    c->n_chunks += b.size();
    c->n_bytes += bytes;
    c->reuse_hits++;
    c->reuse_last_level = c->reuse_level;
    if (c->profiling) {
        c->ev_pending.push_back(ev);
        c->pending_symbols_bound.push_back(syms);
    }
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, s));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->xev, 0));
    }
    *done = true;
    return KC_OK;
}

// The deferred level 3's group size for a counting pass over chunks (device_pass splits them into
// batches of batch_bytes / max_chunks): the batches' largest symbol bound fixes the segment
// geometry of every slot (part_plan, level-2 records of level2_record_bytes); a group takes as many
// batches as 90 % of the HBM left beside the level-1 buffers and the skew list (free + the
// partition buffers held now, less 2 GiB) holds level-2 slots for, at most MAX_SEG_GROUP segments
// per region.  The pass then runs partitioned when one sweep of the table per group beats the
// direct inserts (use_partitioned's rule with the table's bytes spread over the group), e.g. C5's
// one-GPU job, whose table is too large for a sweep per batch.  KC_DEFER=0: off.
static int plan_deferral_nb(kc_ctx* c, uint64_t nb, uint64_t syms);
static int plan_deferral(kc_ctx* c, const kc_chunk* chunks, size_t n) {
    uint64_t nb = 0, syms = 0, used = 0, cnt = 0;
    for (size_t i = 0; i <= n; i++) {
        const bool end = i == n;
        const uint64_t need = end ? 0 : round_up(chunks[i].len, TILE);
        if (!end && chunks[i].len == 0) continue;
        if (end || used + need > c->batch_bytes || cnt + 1 > c->max_chunks) {
            if (cnt) {
                nb++;
                syms = std::max(syms, used + cnt);
            }
            used = cnt = 0;
        }
        used += need;
        cnt++;
    }
    return plan_deferral_nb(c, nb, syms);
}
// (nb batches of at most syms symbols each)
static int plan_deferral_nb(kc_ctx* c, uint64_t nb, uint64_t syms) {
    // KC_DEFER: 0 = off, N = groups of at most N batches (tests)
    const char* kd = std::getenv("KC_DEFER");
    const uint64_t kmax = kd ? std::strtoull(kd, nullptr, 10) : ~0ULL;
    if (kmax == 0 || !c->nbuckets || !c->seg_ok) {
        if (debug_on()) std::fprintf(stderr, "deferred level 3: off (knob %d, table %d, segmented levels %d)\n",
                                     kmax != 0, c->nbuckets != 0, (int)c->seg_ok);
        return KC_OK;
    }
    const PathKnob pk = insert_path_knob();
    if (pk == PathKnob::Direct || pk == PathKnob::Exact) return KC_OK;
    if (nb < 2) return KC_OK;
    const PartPlan p = part_plan(c, syms, true, table_geo(c), 0, 1, 0, true);
    if (p.cap1 == 0) {
        if (debug_on()) std::fprintf(stderr, "deferred level 3: off (exact layout for this batch size)\n");
        return KC_OK;
    }
    const uint64_t rec2 = level2_record_bytes(c->W, c->cfg.k, c->R);
    const double slot_bytes = (double)c->R * p.B2 * p.cap2 * rec2;
    size_t fr = 0, tot = 0;
    HIPCHK(c, hipMemGetInfo(&fr, &tot));
    const double held = (double)(c->k1_words + c->k2_words + c->spill_words) * 8.0;
    const double fixed = (double)(std::max(p.need1, c->k1_words) + std::max(p.spill_words, c->spill_words)) * 8.0;
    const double avail = 0.9 * ((double)fr + held - fixed) - (double)(2ull << 30);
    uint64_t g = avail > 0 ? (uint64_t)(avail / slot_bytes) : 0;
    g = std::min<uint64_t>({g, kmax, nb, MAX_SEG_GROUP / std::max<uint32_t>(1, p.B2),
                            ((1ULL << 31) - 1) / ((uint64_t)p.B2 * p.cap2)});
    // per batch: the direct inserts against the levels' key traffic + the group's table sweep
    const double table_bytes = (double)c->nbuckets * 128.0;
    const bool part_wins = pk == PathKnob::Partitioned || use_partitioned(c, syms) ||
                           (g >= 2 && (double)syms * 275.0 > (double)syms * (4.0 * c->W + 1) * 8.0 +
                                                                  2.0 * table_bytes / (double)g);
    if (debug_on())
        std::fprintf(stderr,
                     "deferred level 3: %llu batches, slot %.2f GB (%llu-byte records), free %.1f GB -> groups of "
                     "%llu%s\n",
                     (unsigned long long)nb, slot_bytes / 1e9, (unsigned long long)rec2, fr / 1e9,
                     (unsigned long long)g, part_wins ? "" : " (direct inserts cheaper: off)");
    if (g < 2 || !part_wins) return KC_OK;
    c->defer_on = true;
    c->defer_g = (uint32_t)g;
    c->defer_syms = syms;
    return KC_OK;
}

// Every exit of a pass (an error inside it included) ends its deferral; an error that leaves a
// group's batches counted without their level 3 marks the job broken
struct DeferEnd {
    kc_ctx* c;
    ~DeferEnd() {
        if (c->defer_on && c->defer_n > 0 && c->broken.empty())
            c->broken = "a counting pass failed with " + std::to_string(c->defer_n) +
                        " batch(es) of a deferred group not inserted: " + c->err;
        c->defer_on = c->defer_last = false;
        c->defer_n = 0;
        c->skew_prev = c->heavy_prev = 0;
    }
};

static int device_pass(kc_ctx* c, const uint8_t* img, const kc_chunk* chunks, size_t n, int fmt, int pass,
                       hipStream_t s) {
    if (fmt != KC_FMT_FASTA && fmt != KC_FMT_FASTQ && fmt != KC_FMT_PLAIN) return c->fail(KC_ERR_ARG, "unknown format");
    int rc = flush_host(c);  // keep order with staged host chunks
    if (rc) return rc;
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->xev, 0));
    }
    std::vector<ChunkDesc> batch;
    uint64_t used = 0;
    // one staging batch holds the whole image?  (every chunk is checked before any is counted: a
    // pass either fails before its first batch or runs to its end)
    bool single = false;
    {
        uint64_t tot = 0, cnt = 0;
        for (size_t i = 0; i < n; i++)
            if (chunks[i].len) {
                if (round_up(chunks[i].len, TILE) > c->batch_bytes)
                    return c->fail(KC_ERR_ARG, "chunk larger than the staging batch");
                tot += round_up(chunks[i].len, TILE);
                cnt++;
            }
        single = cnt > 0 && tot <= c->batch_bytes && cnt <= c->max_chunks;
    }
    DeferEnd defer_end{c};
    // level-1 reuse: the Bloom pass keeps its level-1 output if it is the job's only batch
    const bool keep = pass == 1 && c->bloom_batches == 0 && reuse_enabled() && single;
    // the estimate pass's tokenized batches (kc_estimate_distinct_device), if this counting pass reads
    // the same image, chunks and format: used once, then dropped
    bool use_kept = false;
    if (c->kept_valid && pass == 0 && img == c->kept_img && fmt == c->kept_fmt && n == c->kept_chunks.size()) {
        use_kept = true;
        for (size_t i = 0; i < n && use_kept; i++)
            use_kept = chunks[i].off == c->kept_chunks[i].off && chunks[i].len == c->kept_chunks[i].len &&
                       chunks[i].broken_header == c->kept_chunks[i].broken_header;
    }
    if (pass != 3) c->kept_valid = false;
    size_t kept_i = 0;
    // (a pass over kept batches sizes its partition levels for their windows per symbol)
    struct Density {
        kc_ctx* c;
        double d;
        ~Density() { c->win_density = d; }
    } restore_density{c, c->win_density};
    if (use_kept) c->win_density = c->kept_density;
    // a counting pass of several batches defers level 3 (kc_ctx defer_*) when the segmented levels
    // run and HBM holds at least two batches' level-2 segments beside everything else
    c->defer_on = false;
    c->defer_n = 0;
    c->skew_prev = c->heavy_prev = 0;
    if (pass == 0 && !single) {
        rc = plan_deferral(c, chunks, n);
        if (rc) return rc;
    }
    bool last = false;
    auto launch = [&]() -> int {
        if (batch.empty()) return KC_OK;
        // descriptors go through the (idle) pinned desc buffer of the current slot
        std::memcpy(c->h_desc[c->cur], batch.data(), batch.size() * sizeof(ChunkDesc));
        HIPCHK(c, hipMemcpyAsync(c->d_chunks, c->h_desc[c->cur], batch.size() * sizeof(ChunkDesc),
                                 hipMemcpyHostToDevice, s));
        HIPCHK(c, hipEventRecord(c->h_free[c->cur], s));
        hipEvent_t e0 = nullptr, e1 = nullptr;
        const bool timed = c->profiling && pass != 3 && pass != 4;  // (the sketch / routing passes are not timed)
        if (timed) {
            e0 = c->get_event();
            e1 = c->get_event();
            HIPCHK(c, hipEventRecord(e0, s));
        }
        // the image is tokenized in place (no gather into the stage): "gather" is ~0
        if (timed) HIPCHK(c, hipEventRecord(e1, s));
        // the checksum of a batch the Bloom pass may keep (what a counting pass must present
        // again) runs on a second stream beside the pass's levels: both only read the image
        // (C3: 0.31 ms of streaming hidden under the latency-bound level 1)
        if (keep) {
            if (!c->aux) {
                HIPCHK(c, hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
                for (auto& e : c->aev) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
            }
            uint64_t max_len = 0;
            for (auto& d : batch) max_len = std::max<uint64_t>(max_len, d.len);
            HIPCHK(c, hipEventRecord(c->aev[0], s));
            HIPCHK(c, hipStreamWaitEvent(c->aux, c->aev[0], 0));
            HIPCHK(c, launch_checksum(img, c->d_chunks, (int)batch.size(), max_len, c->d_sum, c->aux));
            HIPCHK(c, hipEventRecord(c->aev[1], c->aux));
        }
        // the host gate of the batch's tail (the call waits for the batch) only for a one-batch
        // image; the batches of a larger image keep the device gate (kc_api.h: kc_count_device)
        // -- or a deferred pass, which reads each batch's flags
        c->defer_last = last;
        int r;
        if (use_kept && kept_i < c->kept.size()) {
            const PackedView kv{c->keep_pk + c->kept[kept_i].first, c->keep_bk + c->kept[kept_i].first};
            r = run_batch(c, img, c->kept[kept_i].second, 0, fmt, pass, s, e0, e1, keep, single, &kv,
                          c->d_kept_len + kept_i);
            kept_i++;
        } else {
            r = run_batch(c, img, used, batch.size(), fmt, pass, s, e0, e1, keep, single);
        }
        if (keep) HIPCHK(c, hipStreamWaitEvent(s, c->aev[1], 0));  // (before an error return, too)
        if (r) return r;
        if (keep && c->reuse_kept) {
            c->reuse_img = img;
            c->reuse_chunks = batch;
            c->reuse_fmt = fmt;
            c->reuse_used = used;
        }
        HIPCHK(c, hipEventSynchronize(c->h_free[c->cur]));
        batch.clear();
        used = 0;
        return KC_OK;
    };
    for (size_t i = 0; i < n; i++) {
        const uint64_t need = round_up(chunks[i].len, TILE);
        if (chunks[i].len == 0) continue;
        if (used + need > c->batch_bytes || batch.size() + 1 > c->max_chunks) {
            rc = launch();
            if (rc) return rc;
        }
        ChunkDesc d;
        d.src_off = chunks[i].off;
        d.stage_off = used;
        d.len = chunks[i].len;
        d.bh = chunks[i].broken_header ? 1 : 0;
        d.pad = 0;
        batch.push_back(d);
        used += need;
        if (pass == 0) { c->n_chunks++; c->n_bytes += chunks[i].len; }
    }
    last = true;
    rc = launch();
    if (rc) return rc;
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, s));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->xev, 0));
    }
    return KC_OK;
}

// ------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------
extern "C" {

const char* kc_last_error(const kc_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

int kc_create(const kc_config* cfg, kc_ctx** out) {
    if (!cfg || !out) { g_create_error = "null argument"; return KC_ERR_ARG; }
    *out = nullptr;
    if (cfg->k < 1 || cfg->k > KC_MAX_K) {
        g_create_error = "k must be in 1.." + std::to_string(KC_MAX_K);
        return KC_ERR_ARG;
    }
    static_assert(KC_MAX_K == MAX_K, "include/kc_api.h and kc_internal.h agree on the largest k");
    if (cfg->mode < 0 || cfg->mode > 2) { g_create_error = "mode must be 0, 1 or 2"; return KC_ERR_ARG; }
    if (cfg->bf_enable && (cfg->est_unique == 0 || !(cfg->fpr >= 0.001 && cfg->fpr <= 0.999))) {
        g_create_error = "bloom filter needs est_unique > 0 and 0.001 <= fpr <= 0.999";
        return KC_ERR_ARG;
    }
    kc_ctx* c = new kc_ctx();
    c->cfg = *cfg;
    if (const char* v = std::getenv("KC_STRICT_CAPACITY")) c->strict_capacity = std::atoi(v) != 0;
    c->W = words_for_k(cfg->k);
    c->S = slots_per_bucket(c->W);
    auto bail = [&](int code, const std::string& m) {
        g_create_error = m.empty() ? c->err : m;
        kc_destroy(c);
        return code;
    };
    hipError_t e = hipSetDevice(cfg->device);
    if (e != hipSuccess) return bail(KC_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
    uint64_t batch = cfg->batch_bytes;
    if (!batch) {
        // Every staged batch of the partitioned insert sweeps the table once, so batches are
        // as large as the device allows: the partition buffers take ~28 W + 4 bytes per
        // staged byte (two segmented key buffers, the skew lists, the packed stream); use ~40 % of free
        // HBM, within [256 MiB, 2 GiB] (the pinned host stage is two batches).
        size_t fr = 0, tot = 0;
        batch = kDefaultBatch;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess)
            batch = std::min<uint64_t>(2ull << 30, std::max<uint64_t>(kDefaultBatch,
                                                                       (uint64_t)(0.4 * fr) / (28 * c->W + 4)));
    }
    c->batch_bytes = round_up(batch, TILE);
    c->max_chunks = c->batch_bytes / TILE;
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess)
        return bail(KC_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
    for (int i = 0; i < 2; i++) {  // (the pinned byte stages are allocated on first host chunk)
        if (hipHostMalloc(&c->h_desc[i], c->max_chunks * sizeof(ChunkDesc), hipHostMallocDefault) != hipSuccess)
            return bail(KC_ERR_NOMEM, "pinned staging allocation failed");
        if (hipEventCreateWithFlags(&c->h_free[i], hipEventDisableTiming) != hipSuccess)
            return bail(KC_ERR_HIP, "event creation failed");
    }
    if (hipEventCreateWithFlags(&c->xev, hipEventDisableTiming) != hipSuccess)
        return bail(KC_ERR_HIP, "event creation failed");
    const uint64_t ntiles = c->batch_bytes / TILE;
    if (hipMalloc(&c->d_pk, ((c->batch_bytes + c->max_chunks) / 32 + 4) * 8) != hipSuccess ||
        hipMalloc(&c->d_bk, ((c->batch_bytes + c->max_chunks) / 32 + 4) * 4) != hipSuccess ||
        hipMalloc(&c->d_tiles, ntiles * sizeof(TileInfo)) != hipSuccess ||
        hipMalloc(&c->d_touts, ntiles * sizeof(TileOut)) != hipSuccess ||
        hipMalloc(&c->d_tblk, (ntiles / 1024 + 2) * sizeof(TileOut)) != hipSuccess ||
        hipMalloc(&c->d_chunks, c->max_chunks * sizeof(ChunkDesc)) != hipSuccess ||
        hipMalloc(&c->d_ctr, sizeof(DevCounters)) != hipSuccess ||
        hipMalloc(&c->d_sum, 2 * CHECKSUM_SLOTS * sizeof(unsigned long long)) != hipSuccess)
        return bail(KC_ERR_NOMEM, "device staging allocation failed");
    if (hipMemsetAsync(c->d_ctr, 0, sizeof(DevCounters), c->stream) != hipSuccess)
        return bail(KC_ERR_HIP, "memset failed");
    if (cfg->bf_enable) {
        bloom_sizes(cfg->est_unique, cfg->fpr, &c->bf_bits, &c->nh, &c->nh_gate);
        if (c->nh > MAX_NH) return bail(KC_ERR_ARG, "too many Bloom hash functions");
        if (bloom_blocks(c->bf_bits) > (1ULL << 32)) return bail(KC_ERR_ARG, "Bloom filter too large (-u)");
        const char* lay = std::getenv("KC_BLOOM_LAYOUT");
        c->bloom_blocked = !(lay && !std::strcmp(lay, "reference"));
        const uint64_t words = bloom_words(c);
        if (hipMalloc(&c->d_bloom, words * 4) != hipSuccess)
            return bail(KC_ERR_NOMEM, "Bloom filter allocation failed");
        if (hipMemsetAsync(c->d_bloom, 0, words * 4, c->stream) != hipSuccess) return bail(KC_ERR_HIP, "memset");
        c->bloom_fresh = true;
        if (c->bloom_blocked) {
            // filter regions of up to BF_BLOCKS_PER_REGION (1024) blocks = 64 KiB, F1 x F2 as
            // for the table (all powers of two here)
            const uint64_t nb = bloom_blocks(c->bf_bits);
            const uint64_t R = std::max<uint64_t>(1, nb / BF_BLOCKS_PER_REGION);
            int rbits = 0;
            while ((1ULL << rbits) < R) rbits++;
            const int f1bits = std::min(10, (rbits + 1) / 2);
            c->bgeo.R = R;
            c->bgeo.f2bits = rbits - f1bits;
            c->bgeo.F2 = 1u << c->bgeo.f2bits;
            c->bgeo.F1 = (uint32_t)(R >> c->bgeo.f2bits);
            c->bgeo.W = 1;
            // partition reuse: fine bins for a table of up to 2 * est_unique slots (the table
            // of the counting pass holds 2 * new_in_second <= about 2 * -u), never coarser than
            // the filter regions, and as fine as level 1 (two workgroups per CU), level 2 and
            // k_b3 (segments per filter region) allow
            {
                uint64_t want = std::max<uint64_t>(2 * cfg->est_unique, 64);
                want += want / 4;
                const uint64_t regions = std::max<uint64_t>(1, ((want + c->S - 1) / c->S + BPR - 1) / BPR);
                int fb = rbits, f1 = 0;
                while ((1ULL << fb) < regions) fb++;
                // (wide keys run one level-1 workgroup per CU anyway)
                const size_t p1_cap = p1_lds_bytes(c->W, 1) <= 80 * 1024 ? 80 * 1024 : 160 * 1024;
                for (; fb >= rbits; fb--) {
                    f1 = std::min(fb, std::min(8, (fb + 1) / 2 + 1));
                    while (f1 > 0 && p1_lds_bytes(c->W, 1u << f1) > p1_cap) f1--;
                    const uint32_t F2 = 1u << (fb - f1), F1 = 1u << f1;
                    const uint32_t B2 = std::max<uint32_t>(1, std::min<uint32_t>(64, 2048 / F1));
                    // (budgeted at 32 bytes per level-2 bin, as before the scatter's bins
                    // took 24: the finer bins that now fit, F2 = 1024 at C3's -u, measured
                    // slower, 29.0 vs 31-32 G k-mers/s, profiles/r02_v15_bench.json)
                    if (p2f_lds_bytes(c->W, F2, 2048 / B2 + 1) + (size_t)F2 * 8 <= 160 * 1024 &&
                        (1ULL << (fb - rbits)) * B2 <= MAX_SEG_GROUP)
                        break;
                }
                if (fb >= rbits) {
                    c->fgeo_max_R = 1ULL << fb;
                    // the job starts at no more than 2^16 fine bins: -u usually overstates the
                    // k-mers that pass the gate (C3: -u 4e8 for 50 M), and level 2's 256-bin
                    // scatter of C2's table is the fastest shape
                    while (fb > rbits && (1ULL << fb) > (1ULL << 16)) fb--;
                    f1 = std::min(fb, std::min(8, (fb + 1) / 2 + 1));
                    while (f1 > 0 && p1_lds_bytes(c->W, 1u << f1) > p1_cap) f1--;
                    c->fgeo.R = 1ULL << fb;
                    c->fgeo.f2bits = fb - f1;
                    c->fgeo.F2 = 1u << c->fgeo.f2bits;
                    c->fgeo.F1 = 1u << f1;
                    c->fgeo.W = c->W;
                }
            }
        }
    } else {
        int rc = alloc_table(c, cfg->table_slots);
        if (rc) return bail(rc, "");
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) return bail(KC_ERR_HIP, "stream sync failed");
    *out = c;
    return KC_OK;
}

void kc_destroy(kc_ctx* c) {
    if (!c) return;
    if (c->stream) hipStreamSynchronize(c->stream);
    for (int i = 0; i < 2; i++) {
        if (c->h_stage[i]) hipHostFree(c->h_stage[i]);
        if (c->h_desc[i]) hipHostFree(c->h_desc[i]);
        if (c->h_free[i]) hipEventDestroy(c->h_free[i]);
    }
    hipFree(c->d_stage);
    hipFree(c->d_pk);
    hipFree(c->d_bk);
    hipFree(c->d_tiles);
    hipFree(c->d_touts);
    hipFree(c->d_tblk);
    hipFree(c->d_chunks);
    hipFree(c->d_ctr);
    hipFree(c->d_sum);
    hipFree(c->d_hll);
    hipFree(c->d_skm);
    hipFree(c->keep_pk);
    hipFree(c->keep_bk);
    hipFree(c->d_kept_len);
    hipFree(c->d_kept_win);
    hipFree(c->d_cwords);
    hipFree(c->d_csecond);
    hipFree(c->d_cstat);
    hipFree(c->d_keep_fill);
    hipFree(c->d_keep_fill2);
    hipFree(c->d_table);
    hipFree(c->d_bloom);
    hipFree(c->pb.hist1);
    hipFree(c->pb.off1);
    hipFree(c->pb.hist2);
    hipFree(c->pb.off2);
    hipFree(c->pb.bsum);
    hipFree(c->d_keys1);
    hipFree(c->d_keys2);
    hipFree(c->d_spill);
    hipFree(c->d_gstart);
    hipFree(c->d_mstart);
    hipFree(c->d_mlen);
    hipFree(c->pbf.hist1);
    hipFree(c->pbf.off1);
    hipFree(c->pbf.hist2);
    hipFree(c->pbf.off2);
    hipFree(c->pbf.bsum);
    hipFree(c->d_rhist);
    hipFree(c->d_roff);
    hipFree(c->d_rbsum);
    if (c->xev) hipEventDestroy(c->xev);
    for (auto e : c->aev)
        if (e) hipEventDestroy(e);
    if (c->aux) hipStreamDestroy(c->aux);
    for (auto e : c->ev_pool) hipEventDestroy(e);
    for (auto& ev : c->ev_pending)
        for (auto e : ev)
            if (e) hipEventDestroy(e);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

int kc_bloom_chunk(kc_ctx* c, const uint8_t* buf, size_t len, int fmt, int bh) {
    if (!c) return KC_ERR_ARG;
    JOB_OK(c);
    if (!c->cfg.bf_enable || c->bloom_final) return c->fail(KC_ERR_STATE, "bloom pass not active");
    return add_host_chunk(c, buf, len, fmt, bh, 1);
}

int kc_bloom_device(kc_ctx* c, const uint8_t* img, const kc_chunk* chunks, size_t n, int fmt, void* s) {
    if (!c || (!img && n) || (!chunks && n)) return KC_ERR_ARG;
    JOB_OK(c);
    if (!c->cfg.bf_enable || c->bloom_final) return c->fail(KC_ERR_STATE, "bloom pass not active");
    return device_pass(c, img, chunks, n, fmt, 1, pick_stream(c, s));
}

int kc_bloom_finalize(kc_ctx* c, uint64_t* new_in_second) {
    if (!c) return KC_ERR_ARG;
    if (!c->cfg.bf_enable || c->bloom_final) return c->fail(KC_ERR_STATE, "bloom pass not active");
    int rc = flush_host(c);
    if (rc) return rc;
    HIPCHK(c, hipDeviceSynchronize());
    DevCounters h;
    HIPCHK(c, hipMemcpy(&h, c->d_ctr, sizeof(h), hipMemcpyDeviceToHost));
    if (new_in_second) *new_in_second = h.new_in_second;
    c->bloom_final = true;
    // partition reuse: the only Bloom batch kept its partitions and no key of them went to a
    // skew list.  The table then takes power-of-two hash-prefix bins: R_t regions with the
    // fine geometry's coarse bins (F1); from level 2 if its regions are unions of fine bins
    // (R_t <= R_fine, at most MAX_SEG_GROUP segments per region), else from level 1 if that
    // level 2 fits the LDS.
    bool reuse = c->reuse_kept && c->bloom_batches == 1 && h.part_fallbacks == 0 && h.spilled == 0 && h.heavy == 0;
    const uint64_t slots = 2 * h.new_in_second;  // main.cpp:454
    c->reuse_level = 0;
    if (reuse) {
        uint64_t want = std::max<uint64_t>(slots, 64);
        want += want / 4;
        const uint64_t regions = std::max<uint64_t>(1, ((want + c->S - 1) / c->S + BPR - 1) / BPR);
        uint64_t rt = c->fgeo.F1;
        while (rt < regions) rt *= 2;
        const uint32_t nseg = (c->pbf.nblk1 + c->pbf.B2 - 1) / std::max<uint32_t>(1, c->pbf.B2);
        if (rt <= c->fgeo.R && (c->fgeo.R / rt) * c->pbf.B2 <= MAX_SEG_GROUP)
            c->reuse_level = 2;
        else if (p2f_lds_bytes(c->W, (uint32_t)(rt / c->fgeo.F1), nseg) <= 160 * 1024 && rt < (1ULL << 32))
            c->reuse_level = 1;
        reuse = c->reuse_level != 0;
        // adaptive fine geometry for the context's next job (kc_reset applies it): fine
        // bins as coarse as the table regions just sized, so that a level-2 region is one
        // fine bin (one segment group per k_p3 workgroup, fewer and fuller level-2 bins:
        // C3 31.3 -> 29.4 ms, profiles/r03_ab_fb16.txt); back to the create-time geometry
        // when this job's table outgrew the learned one.  The first job keeps the default.
        const uint64_t floor_r = std::max<uint64_t>(c->bgeo.R, c->fgeo.F1);
        if (c->reuse_level == 2)
            c->fgeo_next_R = std::max(rt, floor_r);
        else if (rt > c->fgeo.R && c->fgeo.R < c->fgeo_max_R)
            c->fgeo_next_R = c->fgeo_max_R;
    }
    if (reuse) {
        unsigned long long part[CHECKSUM_SLOTS];
        HIPCHK(c, hipMemcpy(part, c->d_sum, sizeof(part), hipMemcpyDeviceToHost));
        c->reuse_sum = 0;
        for (auto v : part) c->reuse_sum += v;
        c->reuse_windows = h.bf_windows;
    }
    c->reuse_ok = reuse;
    if (debug_on())
        std::fprintf(stderr, "reuse finalize: kept %d batches %d fallbacks %llu spilled %llu heavy %llu -> level %d\n",
                     (int)c->reuse_kept, c->bloom_batches, (unsigned long long)h.part_fallbacks,
                     (unsigned long long)h.spilled, (unsigned long long)h.heavy, c->reuse_level);
    rc = alloc_table(c, slots, reuse ? c->fgeo.F1 : 0);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return KC_OK;
}

int kc_count_chunk(kc_ctx* c, const uint8_t* buf, size_t len, int fmt, int bh) {
    if (!c) return KC_ERR_ARG;
    JOB_OK(c);
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "kc_bloom_finalize must precede the counting pass");
    return add_host_chunk(c, buf, len, fmt, bh, 0);
}

int kc_count_device(kc_ctx* c, const uint8_t* img, const kc_chunk* chunks, size_t n, int fmt, void* s) {
    if (!c || (!img && n) || (!chunks && n)) return KC_ERR_ARG;
    JOB_OK(c);
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "kc_bloom_finalize must precede the counting pass");
    if (c->reuse_ok) {  // one chance: the first counting pass after the Bloom pass
        c->reuse_ok = false;
        bool done = false;
        const int rc = count_reused(c, img, chunks, n, fmt, pick_stream(c, s), &done);
        if (rc || done) return rc;
    }
    return device_pass(c, img, chunks, n, fmt, 0, pick_stream(c, s));
}

int kc_estimate_distinct_device(kc_ctx* c, const uint8_t* img, const kc_chunk* chunks, size_t n, int fmt, void* sp,
                                double* estimate) {
    if (!c || !estimate || (!img && n) || (!chunks && n)) return KC_ERR_ARG;
    hipStream_t s = pick_stream(c, sp);
    if (!c->d_hll && hipMalloc(&c->d_hll, HLL_M * 4) != hipSuccess)
        return c->fail(KC_ERR_NOMEM, "sketch allocation failed");
    HIPCHK(c, hipMemsetAsync(c->d_hll, 0, HLL_M * 4, s));
    // the tokenized batches are kept for the counting pass when they take < 1/8 of the free HBM
    c->kept_valid = false;
    c->kept.clear();
    c->keep_woff = 0;
    c->keep_target = false;
    {
        uint64_t words = 64;
        for (size_t i = 0; i < n; i++) words += (round_up(chunks[i].len, TILE) + 1) / 32 + 5;
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
            if (words > c->keep_cap && (double)words * 12 < (double)(fr + c->keep_cap * 12) / 8) {
                hipFree(c->keep_pk);
                hipFree(c->keep_bk);
                c->keep_pk = nullptr;
                c->keep_bk = nullptr;
                c->keep_cap = 0;
                if (hipMalloc(&c->keep_pk, words * 8) == hipSuccess && hipMalloc(&c->keep_bk, words * 4) == hipSuccess)
                    c->keep_cap = words;
            }
            if (!c->d_kept_len && hipMalloc(&c->d_kept_len, 8192 * 8) == hipSuccess &&
                hipMalloc(&c->d_kept_win, 8192 * 8) == hipSuccess)
                c->kept_len_cap = 8192;
            c->keep_target = c->keep_cap >= words && c->kept_len_cap > 0;
        }
    }
    HIPCHK(c, hipMemsetAsync(&c->d_ctr->est_windows, 0, 8, s));
    int rc = device_pass(c, img, chunks, n, fmt, 3, s);
    const bool kept = c->keep_target;
    c->keep_target = false;
    if (rc) return rc;
    if (kept) {
        // the kept batches' windows per symbol: the counting pass sizes its segments for them (a batch
        // of 150 bp reads holds 0.62 windows per symbol at k = 51; sized per symbol, C4's deferred
        // level-2 slots were 2.1 x its records and a pass took two groups)
        std::vector<uint64_t> wins(c->kept.size()), lens(c->kept.size());
        HIPCHK(c, hipMemcpyAsync(wins.data(), c->d_kept_win, wins.size() * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipMemcpyAsync(lens.data(), c->d_kept_len, lens.size() * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        double d = 0;
        for (size_t i = 0; i < wins.size(); i++) {
            const uint64_t w = wins[i] - (i ? wins[i - 1] : 0);
            d = std::max(d, (double)w / (double)std::max<uint64_t>(1, lens[i]));
        }
        c->kept_density = std::min(1.0, d * 1.02 + 0.005);
        c->kept_valid = true;
        c->kept_img = img;
        c->kept_fmt = fmt;
        c->kept_chunks.assign(chunks, chunks + n);
    }
    std::vector<uint32_t> reg(HLL_M);
    HIPCHK(c, hipMemcpyAsync(reg.data(), c->d_hll, HLL_M * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    // Flajolet et al. 2007: E = alpha_m m^2 / sum 2^-M[j]; linear counting m ln(m / V) below
    // 2.5 m when V registers are empty (a 64-bit hash needs no large-range correction)
    double sum = 0;
    uint32_t zeros = 0;
    for (uint32_t v : reg) {
        sum += std::ldexp(1.0, -(int)v);
        zeros += v == 0;
    }
    const double m = HLL_M, alpha = 0.7213 / (1.0 + 1.079 / m);
    double e = alpha * m * m / sum;
    if (e <= 2.5 * m && zeros) e = m * std::log(m / zeros);
    *estimate = std::ldexp(e, hll_sample_bits(c->W));  // (k_hll_s: the sample's estimate)
    return KC_OK;
}

int kc_size_table(kc_ctx* c, uint64_t slots) {
    if (!c) return KC_ERR_ARG;
    JOB_OK(c);
    if (c->cfg.bf_enable) return c->fail(KC_ERR_STATE, "a Bloom job sizes its table from new_in_second");
    if (!c->table_fresh || c->n_chunks) return c->fail(KC_ERR_STATE, "kc_size_table: the job has counted already");
    int rc = flush_host(c);
    if (rc) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipDeviceSynchronize());  // (the previous job's passes may still read the table)
    const uint64_t phys = slots ? slots : c->cfg.table_slots;
    // a table well below its allocation gives the memory back (the deferred level 3 sizes its
    // groups from free HBM); the same size job after job keeps its allocation
    const uint64_t want = std::max<uint64_t>(phys, 64) + std::max<uint64_t>(phys, 64) / 4;
    const uint64_t bytes = (want + c->S - 1) / c->S * (BUCKET_WORDS * 8) + (uint64_t)BPR * BUCKET_WORDS * 8;
    if (c->d_table && bytes * 4 < c->table_cap_bytes * 3) {
        hipFree(c->d_table);
        c->d_table = nullptr;
        c->table_cap_bytes = 0;
    }
    return alloc_table(c, c->cfg.table_slots, 0, phys);  // (ensure_part re-plans the levels per batch)
}

int kc_route_superkmers_device(kc_ctx* c, const uint8_t* img, const kc_chunk* chunks, size_t n, int fmt,
                               uint32_t nshards, int m, uint64_t* dev_pk, uint32_t* dev_bk, uint64_t cap_words,
                               uint64_t* words, uint64_t* windows, void* sp) {
    if (!c || !words || nshards == 0 || nshards > SKM_MAX_SHARDS || (!img && n) || (!chunks && n)) return KC_ERR_ARG;
    if (cap_words && (!dev_pk || !dev_bk)) return KC_ERR_ARG;
    JOB_OK(c);
    const int mm = m ? m : std::min(SKM_DEFAULT_M, c->cfg.k);
    if (mm < 1 || mm > 32 || mm > c->cfg.k) return c->fail(KC_ERR_ARG, "minimizer length must be in 1..min(32, k)");
    hipStream_t s = pick_stream(c, sp);
    const size_t nw = 2 * SKM_MAX_SHARDS + 16;
    if (!c->d_skm && hipMalloc(&c->d_skm, nw * 8) != hipSuccess)
        return c->fail(KC_ERR_NOMEM, "super-k-mer cursor allocation failed");
    HIPCHK(c, hipMemsetAsync(c->d_skm, 0, nw * 8, s));
    c->skm_shards = nshards;
    c->skm_m = mm;
    c->skm_pk = dev_pk;
    c->skm_bk = dev_bk;
    c->skm_cap = cap_words;
    int rc = device_pass(c, img, chunks, n, fmt, 4, s);
    if (rc) return rc;
    std::vector<unsigned long long> h(nw);
    HIPCHK(c, hipMemcpyAsync(h.data(), c->d_skm, nw * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    uint64_t worst = 0;
    for (uint32_t o = 0; o < nshards; o++) {
        words[o] = h[o];
        if (windows) windows[o] = h[SKM_MAX_SHARDS + o];
        worst = std::max<uint64_t>(worst, h[o]);
    }
    if (cap_words && h[2 * SKM_MAX_SHARDS])
        return c->fail(KC_ERR_NOMEM, "super-k-mer buffer too small: " + std::to_string(worst) +
                                         " words for the largest owner, capacity " + std::to_string(cap_words));
    return KC_OK;
}

// A symbol stream in HBM (a received super-k-mer stream) through the pass's levels in batches of
// about a staging batch's windows, cut at words whose first symbol is a break (no window spans a
// cut), with the deferred level 3 of a counting pass over several batches.
static int packed_pass(kc_ctx* c, const uint64_t* pk, const uint32_t* bk, uint64_t n_words, uint64_t windows, int pass,
                       hipStream_t s) {
    int rc = flush_host(c);  // keep order with staged host chunks
    if (rc) return rc;
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->xev, 0));
    }
    if (n_words == 0) return KC_OK;
    const double nsym = (double)n_words * 32.0;
    const double dens = windows ? std::min(1.0, 1.15 * (double)windows / nsym + 1e-3) : 1.0;
    const uint64_t lim = std::max<uint64_t>(1024, (uint64_t)((double)c->batch_bytes / dens) / 32);
    std::vector<uint64_t> cuts{0};
    std::vector<uint32_t> probe(4096);
    while (n_words - cuts.back() > lim) {
        uint64_t w = cuts.back() + lim;
        bool found = false;
        while (!found && w < n_words) {
            const uint64_t m = std::min<uint64_t>(probe.size(), n_words - w);
            HIPCHK(c, hipMemcpyAsync(probe.data(), bk + w, m * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            uint64_t i = 0;
            while (i < m && !(probe[i] >> 31)) i++;
            w += i;
            found = i < m;
        }
        if (!found) break;
        cuts.push_back(w);
    }
    cuts.push_back(n_words);
    const uint64_t nb = cuts.size() - 1;
    uint64_t maxs = 0;
    for (uint64_t i = 0; i < nb; i++) maxs = std::max<uint64_t>(maxs, (cuts[i + 1] - cuts[i]) * 32);
    struct Density {
        kc_ctx* c;
        double d;
        ~Density() { c->win_density = d; }
    } restore{c, c->win_density};
    c->win_density = dens;
    DeferEnd defer_end{c};
    c->defer_on = false;
    c->defer_n = 0;
    c->skew_prev = c->heavy_prev = 0;
    if (pass == 0 && nb >= 2 && (rc = plan_deferral_nb(c, nb, maxs))) return rc;
    for (uint64_t i = 0; i < nb; i++) {
        c->defer_last = i + 1 == nb;
        const PackedView v{const_cast<uint64_t*>(pk) + cuts[i], const_cast<uint32_t*>(bk) + cuts[i]};
        if ((rc = run_batch(c, nullptr, (cuts[i + 1] - cuts[i]) * 32, 0, 0, pass, s, nullptr, nullptr, false, nb == 1,
                            &v)))
            return rc;
    }
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, s));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->xev, 0));
    }
    return KC_OK;
}

int kc_count_packed_device(kc_ctx* c, const uint64_t* pk, const uint32_t* bk, uint64_t n_words, uint64_t windows,
                           void* sp) {
    if (!c || (n_words && (!pk || !bk))) return KC_ERR_ARG;
    JOB_OK(c);
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "kc_bloom_finalize must precede the counting pass");
    c->reuse_ok = false;  // (the Bloom pass's kept partitions are an image's)
    return packed_pass(c, pk, bk, n_words, windows, 0, pick_stream(c, sp));
}

int kc_bloom_packed_device(kc_ctx* c, const uint64_t* pk, const uint32_t* bk, uint64_t n_words, uint64_t windows,
                           void* sp) {
    if (!c || (n_words && (!pk || !bk))) return KC_ERR_ARG;
    JOB_OK(c);
    if (!c->cfg.bf_enable || c->bloom_final) return c->fail(KC_ERR_STATE, "bloom pass not active");
    return packed_pass(c, pk, bk, n_words, windows, 1, pick_stream(c, sp));
}

int kc_route_device(kc_ctx* c, const uint8_t* img, const kc_chunk* chunks, size_t n, int fmt, uint32_t nshards,
                    uint64_t* dev_out, uint64_t out_capacity, uint64_t* counts, void* sp) {
    if (!c || !counts || !dev_out || nshards == 0 || (!img && n) || (!chunks && n)) return KC_ERR_ARG;
    if (fmt != KC_FMT_FASTA && fmt != KC_FMT_FASTQ && fmt != KC_FMT_PLAIN) return c->fail(KC_ERR_ARG, "unknown format");
    if (c->cfg.bf_enable) return c->fail(KC_ERR_UNSUPPORTED, "sharded counting with the Bloom filter is not supported");
    hipStream_t s = pick_stream(c, sp);
    int rc = flush_host(c);
    if (rc) return rc;
    std::vector<ChunkDesc> batch;
    uint64_t used = 0;
    for (size_t i = 0; i < n; i++) {
        if (!chunks[i].len) continue;
        ChunkDesc d{chunks[i].off, used, chunks[i].len, (uint32_t)(chunks[i].broken_header ? 1 : 0), 0};
        batch.push_back(d);
        used += round_up(chunks[i].len, TILE);
        c->n_chunks++;
        c->n_bytes += chunks[i].len;
    }
    if (used > c->batch_bytes || batch.size() > c->max_chunks)
        return c->fail(KC_ERR_ARG, "kc_route_device: the chunks must fit one staging batch");
    const uint64_t syms = used + batch.size();
    if (out_capacity < syms) return c->fail(KC_ERR_ARG, "kc_route_device: output capacity too small");
    for (uint32_t d = 0; d < nshards; d++) counts[d] = 0;
    if (batch.empty()) return KC_OK;
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->xev, 0));
    }
    rc = ensure_part(c, syms, false, nshards);  // level-1 bins = the shards
    if (rc) return rc;
    if ((uint64_t)nshards * c->pb.nblk1 > c->pb_cap.h1) return c->fail(KC_ERR_ARG, "too many shards");
    std::array<hipEvent_t, 4> ev{};
    if (c->profiling)
        for (auto& e : ev) e = c->get_event();
    if (c->profiling) HIPCHK(c, hipEventRecord(ev[0], s));
    std::memcpy(c->h_desc[c->cur], batch.data(), batch.size() * sizeof(ChunkDesc));
    HIPCHK(c, hipMemcpyAsync(c->d_chunks, c->h_desc[c->cur], batch.size() * sizeof(ChunkDesc), hipMemcpyHostToDevice, s));
    if (c->profiling) HIPCHK(c, hipEventRecord(ev[1], s));
    const PackedView sv{c->d_pk, c->d_bk};
    HIPCHK(c, launch_tokenize(img, used / TILE, c->d_chunks, (int)batch.size(), fmt, c->d_tiles, c->d_touts,
                              c->d_tblk, sv, syms, c->d_ctr, s));
    if (c->profiling) HIPCHK(c, hipEventRecord(ev[2], s));
    HIPCHK(c, launch_route(sv, c->cfg.k, c->W, c->d_ctr, c->pb, nshards, dev_out, s));
    if (c->profiling) {
        HIPCHK(c, hipEventRecord(ev[3], s));
        c->ev_pending.push_back(ev);
    }
    // per-owner totals: off1[d * nblk1], d = 0..nshards (the last one is the total)
    std::vector<uint64_t> offs(nshards + 1);
    for (uint32_t d = 0; d <= nshards; d++)
        HIPCHK(c, hipMemcpyAsync(&offs[d], c->pb.off1 + (uint64_t)d * c->pb.nblk1, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    for (uint32_t d = 0; d < nshards; d++) counts[d] = offs[d + 1] - offs[d];
    return KC_OK;
}

int kc_route_hint(kc_ctx* c, uint32_t nshards) {
    if (!c || nshards > RT_MAX_PARTS) return KC_ERR_ARG;
    int rc = kc_sync(c);  // (the level-3 passes in flight keep the previous pointer)
    if (rc) return rc;
    c->own_parts = nshards;
    return own_prep(c);
}

int kc_route_table_device(kc_ctx* c, uint32_t nshards, uint64_t* dev_out, uint64_t out_capacity, uint64_t* counts,
                          void* sp) {
    if (!c || !counts || nshards == 0 || nshards > 64) return KC_ERR_ARG;
    JOB_OK(c);
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "no table");
    hipStream_t s = pick_stream(c, sp);
    int rc = flush_host(c);
    if (rc) return rc;
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->xev, 0));
    }
    rc = materialize_zero(c, s);
    if (rc) return rc;
    const uint64_t nblk = (c->nbuckets + 255) / 256, n = nshards * nblk;
    rc = route_bufs(c, n);
    if (rc) return rc;
    if (c->own_parts && !c->pb.own_parts) own_prep(c);  // (d_rhist moved: the level-3 passes follow it)
    const TableView tv = table_view(c);
    std::array<hipEvent_t, 4> ev{};
    if (c->profiling) {
        ev[2] = c->get_event();
        ev[3] = c->get_event();
        HIPCHK(c, hipEventRecord(ev[2], s));
    }
    // the level-3 passes kept the per-block counts (kc_route_hint): only their scan runs
    const bool kept = c->own_valid && nshards == c->own_parts && c->pb.own_hist == c->d_rhist;
    HIPCHK(c, launch_route_table(tv, nshards, c->d_rhist, c->d_roff, c->d_rbsum, nullptr, s, kept ? 1 : 0));
    c->route_counts_kept += kept;
    c->own_valid = nshards == c->own_parts && c->pb.own_hist == c->d_rhist;  // (the counts of this table)
    std::vector<uint64_t> offs(nshards + 1);
    for (uint32_t d = 0; d <= nshards; d++)
        HIPCHK(c, hipMemcpyAsync(&offs[d], c->d_roff + d * nblk, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    for (uint32_t d = 0; d < nshards; d++) counts[d] = offs[d + 1] - offs[d];
    if (!dev_out) {  // count only
        for (auto e : ev)
            if (e) c->ev_pool.push_back(e);
        return KC_OK;
    }
    if (out_capacity < offs[nshards])
        return c->fail(KC_ERR_ARG, "kc_route_table_device: output capacity too small (" +
                                       std::to_string(offs[nshards]) + " records)");
    HIPCHK(c, launch_route_table(tv, nshards, c->d_rhist, c->d_roff, c->d_rbsum, dev_out, s));
    if (c->profiling) {
        HIPCHK(c, hipEventRecord(ev[3], s));
        c->ev_pending.push_back(ev);
    }
    HIPCHK(c, hipStreamSynchronize(s));
    return KC_OK;
}

int kc_insert_counts_device(kc_ctx* c, const uint64_t* recs, uint64_t n, void* sp) {
    if (!c || (!recs && n)) return KC_ERR_ARG;
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "no table");
    hipStream_t s = pick_stream(c, sp);
    int rc = flush_host(c);
    if (rc) return rc;
    if (n == 0) return KC_OK;
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->xev, 0));
    }
    std::array<hipEvent_t, 4> ev{};
    if (c->profiling) {
        ev[2] = c->get_event();
        ev[3] = c->get_event();
        HIPCHK(c, hipEventRecord(ev[2], s));
    }
    const bool part = use_partitioned(c, n);
    if (part) {
        rc = ensure_part(c, (n * (c->W + 1) + c->W - 1) / c->W, false);  // records are W + 1 words
        if (rc) return rc;
    }
    if (!part) {
        rc = materialize_zero(c, s);
        if (rc) return rc;
    }
    HIPCHK(c, launch_insert_counts(recs, n, part, table_view(c), c->d_ctr, c->pb, c->table_fresh, s));
    own_after_write(c, false, false);
    c->table_fresh = c->table_zero_pending = false;
    if (c->profiling) {
        HIPCHK(c, hipEventRecord(ev[3], s));
        c->ev_pending.push_back(ev);
    }
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, s));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->xev, 0));
    }
    return KC_OK;
}

int kc_insert_counts_runs_device(kc_ctx* c, const uint64_t* recs, const uint64_t* group_counts, uint32_t ngroups,
                                 void* sp) {
    if (!c || !group_counts || ngroups == 0 || ngroups > 64) return KC_ERR_ARG;
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "no table");
    std::vector<uint64_t> gs(ngroups + 1, 0);
    uint64_t maxn = 0;
    for (uint32_t g = 0; g < ngroups; g++) {
        gs[g + 1] = gs[g] + group_counts[g];
        maxn = std::max(maxn, group_counts[g]);
    }
    const uint64_t n = gs[ngroups];
    if (!recs && n) return KC_ERR_ARG;
    hipStream_t s = pick_stream(c, sp);
    int rc = flush_host(c);
    if (rc) return rc;
    if (n == 0) return KC_OK;
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->xev, 0));
    }
    const uint64_t need = (c->R + 1) * ngroups;
    if (!c->d_gstart && hipMalloc(&c->d_gstart, 65 * 8) != hipSuccess)
        return c->fail(KC_ERR_NOMEM, "merge buffer allocation failed");
    if (need > c->m_cap) {
        hipFree(c->d_mstart);
        hipFree(c->d_mlen);
        c->d_mstart = nullptr;
        c->d_mlen = nullptr;
        c->m_cap = 0;
        if (hipMalloc(&c->d_mstart, need * 8) != hipSuccess || hipMalloc(&c->d_mlen, need * 4) != hipSuccess)
            return c->fail(KC_ERR_NOMEM, "merge buffer allocation failed");
        c->m_cap = need;
    }
    HIPCHK(c, hipMemcpyAsync(c->d_gstart, gs.data(), (ngroups + 1) * 8, hipMemcpyHostToDevice, s));
    // the groups must be sorted by this table's region (a sender table of another geometry,
    // or records not from kc_route_table_device, take the general merge insert)
    unsigned long long* flag = &c->d_ctr->part_overflow;
    HIPCHK(c, hipMemsetAsync(flag, 0, 8, s));
    TableView tv = table_view(c);
    HIPCHK(c, launch_check_runs(recs, c->d_gstart, ngroups, maxn, tv, flag, s));
    unsigned long long unsorted = 0;
    HIPCHK(c, hipMemcpyAsync(&unsorted, flag, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (unsorted) return kc_insert_counts_device(c, recs, n, sp);
    std::array<hipEvent_t, 4> ev{};
    if (c->profiling) {
        ev[2] = c->get_event();
        ev[3] = c->get_event();
        HIPCHK(c, hipEventRecord(ev[2], s));
    }
    HIPCHK(c, launch_insert_counts_runs(recs, c->d_gstart, ngroups, tv, c->d_ctr, c->d_mlen, c->d_mstart,
                                        c->table_fresh, s));
    // records counted like kc_insert_counts_device: inserted += their counts
    own_after_write(c, false, false);
    c->table_fresh = c->table_zero_pending = false;
    if (c->profiling) {
        HIPCHK(c, hipEventRecord(ev[3], s));
        c->ev_pending.push_back(ev);
    }
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, s));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->xev, 0));
    }
    return KC_OK;
}

int kc_bloom_records_device(kc_ctx* c, const uint64_t* recs, uint64_t n, void* sp) {
    if (!c || (!recs && n)) return KC_ERR_ARG;
    if (!c->cfg.bf_enable || c->bloom_final) return c->fail(KC_ERR_STATE, "bloom pass not active");
    if (!c->bloom_blocked) return c->fail(KC_ERR_ARG, "records need the blocked Bloom layout");
    hipStream_t s = pick_stream(c, sp);
    int rc = flush_host(c);
    if (rc) return rc;
    c->bloom_batches++;  // (a Bloom pass of records keeps no partitions)
    c->reuse_kept = false;
    if (n == 0) return KC_OK;
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->xev, 0));
    }
    // exact-layout levels for items of W + 1 words in the filter's region geometry
    const PartGeo g{c->bgeo.F1, c->bgeo.F2, c->bgeo.R, c->W + 1};
    if ((rc = ensure_part_geo(c, n, false, g, c->pbf, c->pbf_cap))) return rc;
    const BloomView bv{c->d_bloom, c->bf_bits ? c->bf_bits - 1 : 0, c->nh, c->nh_gate, c->bloom_blocked,
                       bloom_blocks(c->bf_bits)};
    std::array<hipEvent_t, 4> ev{};
    if (c->profiling) {
        ev[2] = c->get_event();
        ev[3] = c->get_event();
        HIPCHK(c, hipEventRecord(ev[2], s));
    }
    HIPCHK(c, launch_bloom_records(c->W, recs, n, bv, c->bgeo, c->d_ctr, c->pbf, c->bloom_fresh, s));
    c->bloom_fresh = false;
    if (c->profiling) {
        HIPCHK(c, hipEventRecord(ev[3], s));
        c->ev_pending.push_back(ev);
    }
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, s));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->xev, 0));
    }
    return KC_OK;
}

int kc_count_records_device(kc_ctx* c, const uint64_t* recs, uint64_t n, void* sp) {
    if (!c || (!recs && n)) return KC_ERR_ARG;
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "no table (kc_bloom_finalize must precede the counting pass)");
    const bool gate = c->cfg.bf_enable && c->cfg.mode != 1;  // -m 1 -b ignores the filter (main.cpp:482-489)
    if (gate && !c->bloom_blocked) return c->fail(KC_ERR_ARG, "records need the blocked Bloom layout");
    hipStream_t s = pick_stream(c, sp);
    int rc = flush_host(c);
    if (rc) return rc;
    if (n == 0) return KC_OK;
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->xev, 0));
    }
    if ((rc = ensure_part(c, (n * (c->W + 1) + c->W - 1) / c->W, false))) return rc;  // records: W + 1 words
    const BloomView bv{c->d_bloom, c->bf_bits ? c->bf_bits - 1 : 0, c->nh, c->nh_gate, c->bloom_blocked,
                       bloom_blocks(c->bf_bits)};
    std::array<hipEvent_t, 4> ev{};
    if (c->profiling) {
        ev[2] = c->get_event();
        ev[3] = c->get_event();
        HIPCHK(c, hipEventRecord(ev[2], s));
    }
    HIPCHK(c, launch_count_records(c->W, recs, n, table_view(c), bv, c->d_ctr, c->pb, c->table_fresh, gate ? 1 : 0, s));
    own_after_write(c, false, false);
    c->table_fresh = c->table_zero_pending = false;
    if (c->profiling) {
        HIPCHK(c, hipEventRecord(ev[3], s));
        c->ev_pending.push_back(ev);
    }
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, s));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->xev, 0));
    }
    return KC_OK;
}

int kc_insert_keys_device(kc_ctx* c, const uint64_t* keys, uint64_t n, void* sp) {
    if (!c || (!keys && n)) return KC_ERR_ARG;
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "no table");
    hipStream_t s = pick_stream(c, sp);
    int rc = flush_host(c);
    if (rc) return rc;
    if (n == 0) return KC_OK;
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->xev, 0));
    }
    const bool part = use_partitioned(c, n);
    if (part) {
        rc = ensure_part(c, n, false);
        if (rc) return rc;
    }
    std::array<hipEvent_t, 4> ev{};
    if (c->profiling) {
        ev[2] = c->get_event();
        ev[3] = c->get_event();
        HIPCHK(c, hipEventRecord(ev[2], s));
    }
    if (!part) {
        rc = materialize_zero(c, s);
        if (rc) return rc;
    }
    HIPCHK(c, launch_insert_keys(keys, n, part, table_view(c), c->d_ctr, c->pb, c->table_fresh, s));
    own_after_write(c, false, false);
    c->table_fresh = c->table_zero_pending = false;
    if (c->profiling) {
        HIPCHK(c, hipEventRecord(ev[3], s));
        c->ev_pending.push_back(ev);
    }
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, s));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->xev, 0));
    }
    return KC_OK;
}

// the readers of the table (finish, dump, write, compact, ...): the staged work done and a
// deferred reset carried out first
static int sync_for_read(kc_ctx* c) {
    JOB_OK(c);
    int rc = flush_host(c);
    if (rc) return rc;
    rc = materialize_zero(c, c->stream);  // a deferred reset is due before anyone reads the table
    if (rc) return rc;
    HIPCHK(c, hipDeviceSynchronize());
    return KC_OK;
}

// (a deferred reset stays deferred: the next fresh pass writes every region anyway -- the
// sharded merge empties the local table and syncs every step)
int kc_sync(kc_ctx* c) {
    if (!c) return KC_ERR_ARG;
    int rc = flush_host(c);
    if (rc) return rc;
    HIPCHK(c, hipDeviceSynchronize());
    return KC_OK;
}

int kc_finish(kc_ctx* c, kc_stats* st) {
    if (!c) return KC_ERR_ARG;
    int rc = sync_for_read(c);
    if (rc) return rc;
    DevCounters h;
    HIPCHK(c, hipMemcpy(&h, c->d_ctr, sizeof(h), hipMemcpyDeviceToHost));
    if (st) {
        std::memset(st, 0, sizeof(*st));
        st->windows = h.windows;
        st->bf_windows = h.bf_windows;
        st->inserted = h.inserted;
        st->table_slots = c->nbuckets * c->S;
        st->bf_bits = c->bf_bits;
        st->new_in_first = h.new_in_first;
        st->new_in_second = h.new_in_second;
        st->failed_in_first = h.failed_in_first;
        st->chunks = c->n_chunks;
        st->part_fallbacks = h.part_fallbacks;
        st->spilled = h.spilled;
        st->heavy_records = h.heavy;
        st->reused_passes = c->reuse_hits;
        st->reuse_level = (uint64_t)c->reuse_last_level;
        st->route_counts_kept = c->route_counts_kept;
        st->deferred_level3 = c->defer_groups;
        st->bytes = c->n_bytes;
        // occupied slots
        if (c->nbuckets) {
            HIPCHK(c, hipMemsetAsync(&c->d_ctr->occupied, 0, 8, c->stream));
            HIPCHK(c, hipMemsetAsync(&c->d_ctr->dump_n, 0, 8, c->stream));
            TableView tv = table_view(c);
            HIPCHK(c, launch_dump(tv, c->cfg.mode == 0 ? 0 : 1, ~0ULL, nullptr, c->d_ctr, c->stream));
            unsigned long long occ = 0;
            HIPCHK(c, hipMemcpyAsync(&occ, &c->d_ctr->occupied, 8, hipMemcpyDeviceToHost, c->stream));
            HIPCHK(c, hipStreamSynchronize(c->stream));
            st->distinct = occ;
        }
    }
    if (h.invalid)
        return c->fail(KC_ERR_ARG, std::to_string(h.invalid) + " keys passed to kc_insert_keys_device were not table keys "
                                   "(word 0 == 0) and were skipped");
    if (h.overflow) return c->fail(KC_ERR_TABLE_FULL, "Hash table is full (" + std::to_string(h.overflow) +
                                                           " k-mers could not be inserted)");
    if (c->strict_capacity && c->nbuckets) {  // the reference's table: next_prime3mod4(min slots)
        const uint64_t cap = kc_table_size_reference(c->min_slots);
        TableView tv = table_view(c);
        HIPCHK(c, hipMemsetAsync(&c->d_ctr->occupied, 0, 8, c->stream));
        HIPCHK(c, launch_dump(tv, c->cfg.mode == 0 ? 0 : 1, ~0ULL, nullptr, c->d_ctr, c->stream));
        unsigned long long occ = 0;
        HIPCHK(c, hipMemcpyAsync(&occ, &c->d_ctr->occupied, 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (occ > cap)
            return c->fail(KC_ERR_TABLE_FULL, "Hash table is full (" + std::to_string(occ) + " distinct k-mers, the "
                                              "reference's table holds " + std::to_string(cap) + ")");
    }
    return KC_OK;
}

// the compact representation is a snapshot of the table (kc_compact); kc_reset drops it
// The counting passes' key buffers and skew list are scratch that stays allocated between
// batches and jobs (a deferred group holds several batches' level-2 segments: C5 on one GPU,
// ~150 GB).  Before an allocation that would not fit beside them (the compact representation, a
// full dump) they are released; the next counting pass allocates them again (and cannot count
// from a Bloom pass's partitions released this way).
static void make_room(kc_ctx* c, uint64_t bytes) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || (double)fr >= (double)bytes + (double)(1ull << 30)) return;
    if (!c->d_keys1 && !c->d_keys2 && !c->d_spill) return;
    (void)hipDeviceSynchronize();
    hipFree(c->d_keys1);
    hipFree(c->d_keys2);
    hipFree(c->d_spill);
    c->d_keys1 = c->d_keys2 = c->d_spill = nullptr;
    c->k1_words = c->k2_words = c->spill_words = 0;
    c->pb.keys1 = c->pb.keys2 = c->pb.spill = nullptr;
    c->pbf.keys1 = c->pbf.keys2 = c->pbf.spill = nullptr;
    c->reuse_img = nullptr;  // (the kept partitions are gone)
    if (debug_on()) std::fprintf(stderr, "released the partition key buffers for %.1f GB\n", bytes / 1e9);
}

static void drop_compact(kc_ctx* c) {
    hipFree(c->d_cwords);
    hipFree(c->d_csecond);
    c->d_cwords = c->d_csecond = nullptr;
    c->cslots = c->cstarts = c->ckmers = 0;
}

int kc_clear_table(kc_ctx* c) {
    if (!c) return KC_ERR_ARG;
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "no table");
    c->table_zero_pending = true;  // deferred: see materialize_zero
    c->table_fresh = true;
    c->own_valid = false;
    return KC_OK;
}

int kc_reset(kc_ctx* c) {
    if (!c) return KC_ERR_ARG;
    int rc = kc_sync(c);
    if (rc) return rc;
    if (c->d_table) {
        c->table_zero_pending = true;  // deferred: see materialize_zero
        c->table_fresh = true;
        c->own_valid = false;
    }
    if (c->d_bloom) {
        HIPCHK(c, hipMemsetAsync(c->d_bloom, 0, bloom_words(c) * 4, c->stream));
        c->bloom_fresh = true;
        if (c->bloom_final) {  // back to the Bloom pass: the table is sized again after it
            // (its allocation is kept for reuse; ensure_part_geo re-sizes the histograms)
            c->nbuckets = 0;
            c->bloom_final = false;
        }
    }
    HIPCHK(c, hipMemsetAsync(c->d_ctr, 0, sizeof(DevCounters), c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->n_chunks = c->n_bytes = 0;
    c->bloom_batches = 0;
    drop_compact(c);
    c->reuse_kept = c->reuse_ok = false;
    c->reuse_level = 0;
    if (c->fgeo_next_R && c->fgeo_next_R != c->fgeo.R && c->fgeo_next_R <= c->fgeo_max_R) {
        int fb = 0, f1 = 0;
        while ((1ULL << fb) < c->fgeo_next_R) fb++;
        while ((1u << f1) < c->fgeo.F1) f1++;
        c->fgeo.R = 1ULL << fb;
        c->fgeo.f2bits = fb - f1;
        c->fgeo.F2 = 1u << c->fgeo.f2bits;
    }
    c->fgeo_next_R = 0;
    c->reuse_hits = 0;
    c->reuse_last_level = 0;
    c->route_counts_kept = 0;
    c->defer_groups = 0;
    c->defer_n = 0;
    c->skew_prev = c->heavy_prev = 0;
    c->defer_on = c->defer_last = false;
    c->broken.clear();
    c->kept_valid = false;
    return KC_OK;
}

int kc_profile(kc_ctx* c, int enable) {
    if (!c) return KC_ERR_ARG;
    c->profiling = enable != 0;
    return KC_OK;
}

int kc_get_timing(kc_ctx* c, kc_timing* t) {
    if (!c || !t) return KC_ERR_ARG;
    int rc = kc_sync(c);
    if (rc) return rc;
    for (auto& ev : c->ev_pending) {
        float a = 0, b = 0, d = 0;
        if (ev[0]) {  // a full batch: {start, gather, tokenize, count/route}
            HIPCHK(c, hipEventElapsedTime(&a, ev[0], ev[1]));
            HIPCHK(c, hipEventElapsedTime(&b, ev[1], ev[2]));
            c->timing.launches++;
        }
        HIPCHK(c, hipEventElapsedTime(&d, ev[2], ev[3]));  // insert of received keys: {-, -, start, end}
        c->timing.gather_ms += a;
        c->timing.tokenize_ms += b;
        c->timing.count_ms += d;
        for (auto e : ev)
            if (e) c->ev_pool.push_back(e);
    }
    c->ev_pending.clear();
    unsigned long long sl = 0;
    HIPCHK(c, hipMemcpy(&sl, &c->d_ctr->stream_len, 8, hipMemcpyDeviceToHost));
    c->timing.symbols = sl;  // symbols of the LAST batch (exact for single-batch steps)
    *t = c->timing;
    c->timing = kc_timing{};
    return KC_OK;
}

int kc_key_words(const kc_ctx* c) { return c ? c->W : 0; }
void kc_free(void* p) { std::free(p); }

int kc_dump(kc_ctx* c, uint64_t** records, uint64_t* n_records) {
    if (!c || !records || !n_records) return KC_ERR_ARG;
    *records = nullptr;
    *n_records = 0;
    int rc = sync_for_read(c);
    if (rc) return rc;
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "no table");
    TableView tv = table_view(c);
    const int cm = c->cfg.mode == 0 ? 0 : 1;
    const uint64_t a = c->cfg.min_abundance;
    HIPCHK(c, hipMemsetAsync(&c->d_ctr->dump_n, 0, 16 * 8 * 2, c->stream));  // dump_n + occupied lines
    HIPCHK(c, launch_dump(tv, cm, a, nullptr, c->d_ctr, c->stream));
    unsigned long long n = 0;
    HIPCHK(c, hipMemcpyAsync(&n, &c->d_ctr->dump_n, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const size_t rec = (size_t)(c->W + 1) * sizeof(uint64_t);
    uint64_t* h = (uint64_t*)std::malloc(std::max<size_t>(1, n * rec));
    if (!h) return c->fail(KC_ERR_NOMEM, "host allocation failed");
    if (n) {
        uint64_t* d = nullptr;
        make_room(c, n * rec);
        hipError_t e = hipMalloc(&d, n * rec);
        if (e != hipSuccess) { std::free(h); return c->fail(KC_ERR_NOMEM, "dump buffer allocation failed"); }
        HIPCHK(c, hipMemsetAsync(&c->d_ctr->dump_n, 0, 16 * 8 * 2, c->stream));
        HIPCHK(c, launch_dump(tv, cm, a, d, c->d_ctr, c->stream));
        HIPCHK(c, hipMemcpyAsync(h, d, n * rec, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        hipFree(d);
    }
    *records = h;
    *n_records = n;
    return KC_OK;
}

int kc_output_digest(kc_ctx* c, kc_digest* out) {
    if (!c || !out) return KC_ERR_ARG;
    std::memset(out, 0, sizeof(*out));
    if (c->cfg.min_abundance == 0) return KC_OK;  // no output (parallel_parser.hpp:1536 / 858)
    int rc = sync_for_read(c);
    if (rc) return rc;
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "no table");
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 4 * sizeof(unsigned long long)) != hipSuccess)
        return c->fail(KC_ERR_NOMEM, "digest buffer allocation failed");
    unsigned long long h[4] = {0, 0, 0, 0};
    hipError_t e = hipMemsetAsync(d, 0, sizeof(h), c->stream);
    if (e == hipSuccess)
        e = launch_text_digest(table_view(c), c->cfg.mode == 0 ? 0 : 1, c->cfg.min_abundance, c->cfg.k, d, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    hipFree(d);
    if (e != hipSuccess) return c->fail(KC_ERR_HIP, std::string("output digest: ") + hipGetErrorString(e));
    out->lines = h[0];
    out->count_sum = h[1];
    out->hash_sum = h[2];
    out->hash_xor = h[3];
    return KC_OK;
}

// ------------------------------------------------------------------------------
// Kaarme's compact representation: kc_compact_impl.h
// ------------------------------------------------------------------------------
int kc_compact(kc_ctx* c, double load, kc_compact_info* info) {
    if (!c) return KC_ERR_ARG;
    if (load == 0) load = 0.8;
    if (!(load > 0 && load <= 0.95)) return c->fail(KC_ERR_ARG, "load must be in (0, 0.95]");
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "no table");
    if (c->cfg.mode == 0)
        return c->fail(KC_ERR_UNSUPPORTED, "the compact representation holds Kaarme counts (-m 1/2: 14 bits, "
                                           "saturating at 16383)");
    int rc = sync_for_read(c);
    if (rc) return rc;
    rc = materialize_zero(c, c->stream);
    if (rc) return rc;
    drop_compact(c);
    const TableView tv = table_view(c);
    HIPCHK(c, hipMemsetAsync(&c->d_ctr->occupied, 0, 8, c->stream));
    HIPCHK(c, launch_dump(tv, 1, ~0ULL, nullptr, c->d_ctr, c->stream));
    unsigned long long occ = 0;
    HIPCHK(c, hipMemcpyAsync(&occ, &c->d_ctr->occupied, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint64_t nslots = std::max<uint64_t>(64, (uint64_t)std::ceil((double)occ / load));
    if (nslots >> 38) return c->fail(KC_ERR_ARG, "too many k-mers for 38-bit slot pointers");
    uint64_t *src = nullptr, *second = nullptr, *inv = nullptr;
    if (!c->d_cstat && hipMalloc(&c->d_cstat, 4 * sizeof(unsigned long long)) != hipSuccess)
        return c->fail(KC_ERR_NOMEM, "compact counters");
    make_room(c, nslots * 16 + std::max<uint64_t>(1, occ) * c->W * 8 + c->nbuckets * c->S * 8);
    if (hipMalloc(&c->d_cwords, nslots * 8) != hipSuccess || hipMalloc(&src, nslots * 8) != hipSuccess ||
        hipMalloc(&second, std::max<uint64_t>(1, occ) * c->W * 8) != hipSuccess ||
        hipMalloc(&inv, c->nbuckets * c->S * 8) != hipSuccess) {
        hipFree(src);
        hipFree(second);
        hipFree(inv);
        drop_compact(c);
        return c->fail(KC_ERR_NOMEM, "compact representation allocation failed");
    }
    HIPCHK(c, hipMemsetAsync(c->d_cwords, 0, nslots * 8, c->stream));
    HIPCHK(c, hipMemsetAsync(src, 0xFF, nslots * 8, c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_cstat, 0, 4 * sizeof(unsigned long long), c->stream));
    CompactView cv{c->d_cwords, nslots, src, second, c->d_cstat, inv};
    HIPCHK(c, launch_compact_build(tv, cv, c->cfg.k, c->stream));
    unsigned long long starts = 0;
    HIPCHK(c, hipMemcpyAsync(&starts, c->d_cstat, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(src);
    hipFree(inv);
    // the secondary array at its size (the reference grows it as chains start, :2267-2278)
    if (hipMalloc(&c->d_csecond, std::max<uint64_t>(1, starts) * c->W * 8) != hipSuccess) {
        hipFree(second);
        drop_compact(c);
        return c->fail(KC_ERR_NOMEM, "secondary array allocation failed");
    }
    if (starts) HIPCHK(c, hipMemcpyAsync(c->d_csecond, second, starts * c->W * 8, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(second);
    c->cslots = nslots;
    c->cstarts = starts;
    c->ckmers = occ;
    if (info) {
        info->slots = nslots;
        info->kmers = occ;
        info->chain_starts = starts;
        info->bytes = nslots * 8 + starts * c->W * 8;
        info->table_bytes = c->nbuckets * BUCKET_WORDS * 8;
    }
    return KC_OK;
}

static CompactView compact_view(const kc_ctx* c) {
    return CompactView{c->d_cwords, c->cslots, nullptr, c->d_csecond, c->d_cstat};
}

int kc_compact_dump(kc_ctx* c, uint64_t** records, uint64_t* n_records, uint64_t* max_hops, double* mean_hops) {
    if (!c || !records || !n_records) return KC_ERR_ARG;
    *records = nullptr;
    *n_records = 0;
    if (!c->d_cwords) return c->fail(KC_ERR_STATE, "no compact representation (kc_compact)");
    int rc = sync_for_read(c);
    if (rc) return rc;
    const CompactView cv = compact_view(c);
    const uint64_t a = c->cfg.min_abundance;
    unsigned long long st[4];
    HIPCHK(c, hipMemsetAsync(c->d_cstat, 0, sizeof(st), c->stream));
    HIPCHK(c, launch_compact_dump(c->W, cv, c->cfg.k, a, nullptr, c->d_cstat, c->d_cstat + 1, c->stream));
    HIPCHK(c, hipMemcpyAsync(st, c->d_cstat, sizeof(st), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint64_t n = st[0];
    if (st[3]) return c->fail(KC_ERR_STATE, std::to_string(st[3]) + " compact slots did not reconstruct");
    const size_t rec = (size_t)(c->W + 1) * sizeof(uint64_t);
    uint64_t* h = (uint64_t*)std::malloc(std::max<size_t>(1, n * rec));
    if (!h) return c->fail(KC_ERR_NOMEM, "host allocation failed");
    if (n) {
        uint64_t* d = nullptr;
        make_room(c, n * rec);
        if (hipMalloc(&d, n * rec) != hipSuccess) {
            std::free(h);
            return c->fail(KC_ERR_NOMEM, "dump buffer allocation failed");
        }
        HIPCHK(c, hipMemsetAsync(c->d_cstat, 0, sizeof(st), c->stream));
        HIPCHK(c, launch_compact_dump(c->W, cv, c->cfg.k, a, d, c->d_cstat, c->d_cstat + 1, c->stream));
        HIPCHK(c, hipMemcpyAsync(h, d, n * rec, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipMemcpyAsync(st, c->d_cstat, sizeof(st), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        hipFree(d);
    }
    if (max_hops) *max_hops = st[2];
    if (mean_hops) *mean_hops = n ? (double)st[1] / (double)n : 0.0;
    *records = h;
    *n_records = n;
    return KC_OK;
}

int kc_compact_lookup(kc_ctx* c, const uint64_t* keys, uint64_t n, uint32_t* counts) {
    if (!c || (n && (!keys || !counts))) return KC_ERR_ARG;
    if (!c->d_cwords) return c->fail(KC_ERR_STATE, "no compact representation (kc_compact)");
    if (!n) return KC_OK;
    int rc = sync_for_read(c);
    if (rc) return rc;
    uint64_t* dk = nullptr;
    uint32_t* dc = nullptr;
    if (hipMalloc(&dk, n * c->W * 8) != hipSuccess || hipMalloc(&dc, n * 4) != hipSuccess) {
        hipFree(dk);
        return c->fail(KC_ERR_NOMEM, "lookup buffers");
    }
    HIPCHK(c, hipMemcpyAsync(dk, keys, n * c->W * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_compact_lookup(c->W, compact_view(c), c->cfg.k, dk, n, dc, c->stream));
    HIPCHK(c, hipMemcpyAsync(counts, dc, n * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipFree(dk);
    hipFree(dc);
    return KC_OK;
}

int kc_compact_read(kc_ctx* c, uint64_t* words, uint64_t n_words, uint64_t* second, uint64_t n_second_words) {
    if (!c) return KC_ERR_ARG;
    if (!c->d_cwords) return c->fail(KC_ERR_STATE, "no compact representation (kc_compact)");
    if (n_words > c->cslots || n_second_words > c->cstarts * c->W || (n_words && !words) ||
        (n_second_words && !second))
        return c->fail(KC_ERR_ARG, "more words than the compact representation holds");
    int rc = sync_for_read(c);
    if (rc) return rc;
    if (n_words) HIPCHK(c, hipMemcpy(words, c->d_cwords, n_words * 8, hipMemcpyDeviceToHost));
    if (n_second_words) HIPCHK(c, hipMemcpy(second, c->d_csecond, n_second_words * 8, hipMemcpyDeviceToHost));
    return KC_OK;
}

// Text output formatted on the device (the reference formats on one host
// thread, kmer_hash_table.cpp:4318-4524): k_text_bytes + scan give every TEXT_T-bucket
// block its offset in the text, then pieces of <= KC_TEXT_PIECE bytes are formatted by
// k_text, copied to pinned memory and written while the next piece is formatted
// (64 MiB pieces; KC_TEXT_PIECE overrides, >= 128 KiB so a block always fits).
// Lines come out in table order (the reference's order is unspecified too).
static uint64_t text_piece_bytes() {
    const char* e = std::getenv("KC_TEXT_PIECE");  // tests: force many pieces
    const uint64_t v = e ? std::strtoull(e, nullptr, 10) : 0;
    return v ? std::max<uint64_t>(v, 1ull << 17) : 64ull << 20;
}

int kc_write(kc_ctx* c, const char* path) {
    if (!c || !path) return KC_ERR_ARG;
    if (c->cfg.min_abundance == 0) return KC_OK;  // parallel_parser.hpp:1536 / 858
    int rc = sync_for_read(c);
    if (rc) return rc;
    if (!c->nbuckets) return c->fail(KC_ERR_STATE, "no table");
    const TableView tv = table_view(c);
    const int cm = c->cfg.mode == 0 ? 0 : 1;
    const uint64_t a = c->cfg.min_abundance;
    const uint64_t nblk = (c->nbuckets + TEXT_T - 1) / TEXT_T;
    uint32_t* d_bb = nullptr;
    uint64_t *d_off = nullptr, *d_bsum = nullptr;
    uint8_t* d_txt[2] = {nullptr, nullptr};
    uint8_t* h_txt[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    std::vector<uint64_t> off(nblk + 1);
    std::vector<uint32_t> bb(nblk);
    FILE* f = nullptr;
    auto cleanup = [&]() {
        hipStreamSynchronize(c->stream);
        hipFree(d_bb);
        hipFree(d_off);
        hipFree(d_bsum);
        for (int i = 0; i < 2; i++) {
            hipFree(d_txt[i]);
            if (h_txt[i]) hipHostFree(h_txt[i]);
            if (ev[i]) hipEventDestroy(ev[i]);
        }
        if (f) std::fclose(f);
    };
    auto fail = [&](int code, const std::string& m) {
        cleanup();
        return c->fail(code, m);
    };
#define TXCHK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) return fail(KC_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)
    if (hipMalloc(&d_bb, nblk * 4) != hipSuccess || hipMalloc(&d_off, (nblk + 1) * 8) != hipSuccess ||
        hipMalloc(&d_bsum, ((nblk + 4095) / 4096 + 2) * 8) != hipSuccess)
        return fail(KC_ERR_NOMEM, "text offset allocation failed");
    TXCHK(launch_text_bytes(tv, cm, a, c->cfg.k, d_bb, d_off, d_bsum, c->stream));
    TXCHK(hipMemcpyAsync(off.data(), d_off, (nblk + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    TXCHK(hipMemcpyAsync(bb.data(), d_bb, nblk * 4, hipMemcpyDeviceToHost, c->stream));
    TXCHK(hipStreamSynchronize(c->stream));
    const uint64_t total = off[nblk];
    f = std::fopen(path, "wb");
    if (!f) return fail(KC_ERR_IO, std::string("cannot open ") + path);
    // pieces: maximal runs of blocks whose text fits one piece buffer (a block's text is
    // at most TEXT_T * S * (k + 7) bytes < 128 KiB, so every block fits)
    const uint64_t cap = std::min<uint64_t>(text_piece_bytes(), std::max<uint64_t>(total, 1));
    struct Piece { uint64_t b0, b1; uint32_t lds; };
    std::vector<Piece> pieces;
    for (uint64_t b0 = 0; b0 < nblk;) {
        uint64_t b1 = b0;
        uint32_t mx = 0;
        while (b1 < nblk && off[b1 + 1] - off[b0] <= cap) mx = std::max(mx, bb[b1++]);
        if (b1 == b0) return fail(KC_ERR_STATE, "text block larger than a piece");
        if (off[b1] > off[b0]) pieces.push_back({b0, b1, (mx + 15) & ~15u});
        b0 = b1;
    }
    const int nbuf = pieces.size() > 1 ? 2 : 1;
    for (int i = 0; i < nbuf && !pieces.empty(); i++) {
        if (hipMalloc(&d_txt[i], cap) != hipSuccess || hipHostMalloc(&h_txt[i], cap, hipHostMallocDefault) != hipSuccess)
            return fail(KC_ERR_NOMEM, "text buffer allocation failed");
        TXCHK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    }
    for (size_t i = 0; i <= pieces.size(); i++) {
        if (i < pieces.size()) {  // format piece i while piece i - 1 is written
            const Piece& p = pieces[i];
            const int q = (int)(i % nbuf);
            const uint64_t len = off[p.b1] - off[p.b0];
            TXCHK(launch_text(tv, cm, a, c->cfg.k, p.b0, p.b1 - p.b0, d_off, off[p.b0], d_txt[q], p.lds, c->stream));
            TXCHK(hipMemcpyAsync(h_txt[q], d_txt[q], len, hipMemcpyDeviceToHost, c->stream));
            TXCHK(hipEventRecord(ev[q], c->stream));
        }
        if (i >= 1) {
            const Piece& p = pieces[i - 1];
            const int q = (int)((i - 1) % nbuf);
            const uint64_t len = off[p.b1] - off[p.b0];
            TXCHK(hipEventSynchronize(ev[q]));
            if (std::fwrite(h_txt[q], 1, len, f) != len) return fail(KC_ERR_IO, "write failed");
        }
    }
#undef TXCHK
    const int cl = std::fclose(f);
    f = nullptr;
    cleanup();
    if (cl != 0) return c->fail(KC_ERR_IO, "write failed");
    return KC_OK;
}

}  // extern "C"

// The chunk planner reads the image only around chunk ends (io_worker / read_chunk_from_file,
// parallel_parser.hpp:1246-1285, text_reader.h:93-226): templated over how bytes are read --
// a host pointer, or 64 KiB pages of a device image fetched on demand (kc_plan_chunks_device:
// a 1.6 GB image costs its ~160 chunk ends, not a copy of the image)
struct HostImg {
    const uint8_t* p;
    uint8_t operator[](uint64_t i) const { return p[i]; }
    uint64_t find(uint64_t from, uint8_t c, uint64_t size) const {  // first c at >= from, or size
        const void* q = std::memchr(p + from, c, size - from);
        return q ? (uint64_t)((const uint8_t*)q - p) : size;
    }
};
struct DeviceImg {
    static constexpr uint64_t PAGE = 64 << 10;
    const uint8_t* d;
    uint64_t size;
    std::vector<std::pair<uint64_t, std::vector<uint8_t>>> cache;  // a few pages, most recent last
    bool bad = false;
    uint64_t fetched = 0;
    const std::vector<uint8_t>& page(uint64_t pg) {
        for (size_t i = 0; i < cache.size(); i++)
            if (cache[i].first == pg) return cache[i].second;
        if (cache.size() >= 8) cache.erase(cache.begin());
        const uint64_t off = pg * PAGE, len = std::min(PAGE, size - off);
        std::vector<uint8_t> buf(len);
        if (hipMemcpy(buf.data(), d + off, len, hipMemcpyDeviceToHost) != hipSuccess) bad = true;
        fetched += len;
        cache.emplace_back(pg, std::move(buf));
        return cache.back().second;
    }
    uint8_t operator[](uint64_t i) { return page(i / PAGE)[i % PAGE]; }
    uint64_t find(uint64_t from, uint8_t c, uint64_t sz) {
        while (from < sz) {
            const auto& pg = page(from / PAGE);
            const uint64_t o = from % PAGE;
            const void* q = std::memchr(pg.data() + o, c, pg.size() - o);
            if (q) return from - o + (uint64_t)((const uint8_t*)q - pg.data());
            from += pg.size() - o;
        }
        return sz;
    }
};

template <class Img>
static int plan_chunks_impl(Img& image, uint64_t size, int k, uint64_t chunk_size, int fmt, kc_chunk** out,
                            uint64_t* n_out) {
    if (chunk_size == 0) chunk_size = 10ull << 20;  // main.cpp:387
    std::vector<kc_chunk> v;
    if (fmt == KC_FMT_FASTQ) {
        // FASTQ (extension; the reference rejects it): chunks of whole 4-line records, no
        // overlap (a k-mer never spans records).  A record starts at a line that begins
        // with '@' and whose second next line begins with '+' (a quality line starting
        // with '@' is followed two lines later by a sequence line, never by '+').
        auto line_after = [&](uint64_t p) -> uint64_t {  // start of the line after the one at p
            const uint64_t q = image.find(p, '\n', size);
            return q < size ? q + 1 : size;
        };
        auto is_record = [&](uint64_t p) {
            if (p >= size || image[p] != '@') return false;
            const uint64_t l2 = line_after(line_after(p));
            return l2 < size && image[l2] == '+';
        };
        uint64_t pos = 0;
        while (pos < size) {
            uint64_t end = size;
            if (size - pos > chunk_size) {
                end = 0;
                // last record start in (pos, pos + chunk_size]: walk back over line starts
                for (uint64_t q = pos + chunk_size; q > pos; q--)
                    if (image[q - 1] == '\n' && is_record(q)) { end = q; break; }
                if (!end) {  // one record longer than a chunk: cut after it
                    end = size;
                    for (uint64_t q = line_after(pos); q < size; q = line_after(q))
                        if (is_record(q)) { end = q; break; }
                }
            }
            v.push_back(kc_chunk{pos, end - pos, 0, 0});
            pos = end;
        }
    } else {
    const unsigned char start = fmt == KC_FMT_FASTA ? '>' : 0;
    // io_worker: loop while rem >= k, each chunk min(chunk_size, rem) bytes, then
    // read_chunk_from_file with its k = k-1 (parallel_parser.hpp:1246-1285).
    const int64_t back = (int64_t)k - 1;
    int64_t rem = (int64_t)size;
    uint64_t pos = 0;
    bool bh = false;
    while (rem >= (int64_t)k) {
        const int64_t n = std::min<int64_t>((int64_t)chunk_size, rem);
        auto b = [&](int64_t i) { return image[pos + (uint64_t)i]; };
        kc_chunk ck{pos, (uint64_t)n, bh ? 1 : 0, 0};
        v.push_back(ck);
        int64_t fake = 0;
        if (start) {
            int64_t real = 0, si = n - 1;
            if (start == '>')
                for (; real < back && si >= 0; si--) (b(si) != '\n') ? real++ : fake++;  // text_reader.h:143-150
            if (real != back) break;                                                 // text_reader.h:156-160
            // broken header of the NEXT chunk: scan back from the byte before its start
            bh = true;
            for (int64_t i = n - 1 - back - fake; i >= 0; i--) {  // text_reader.h:164-184
                if (b(i) == start) break;
                if (b(i) == '\n') { bh = false; break; }
            }
        }
        if (rem == n) break;                 // text_reader.h:201-204
        const int64_t adv = n - back - fake;  // seek back (k-1) + fake (text_reader.h:210-220)
        if (adv == 0) break;
        rem -= adv;
        pos += (uint64_t)adv;
    }
    }
    kc_chunk* r = (kc_chunk*)std::malloc(std::max<size_t>(1, v.size()) * sizeof(kc_chunk));
    if (!r) return KC_ERR_NOMEM;
    if (!v.empty()) std::memcpy(r, v.data(), v.size() * sizeof(kc_chunk));
    *out = r;
    *n_out = v.size();
    return KC_OK;
}

extern "C" {

int kc_plan_chunks(const uint8_t* image, uint64_t size, int k, uint64_t chunk_size, int fmt, kc_chunk** out,
                   uint64_t* n_out) {
    if (!out || !n_out || k < 1 || (!image && size)) return KC_ERR_ARG;
    HostImg img{image};
    return plan_chunks_impl(img, size, k, chunk_size, fmt, out, n_out);
}

int kc_plan_chunks_device(const uint8_t* dev_image, uint64_t size, int k, uint64_t chunk_size, int fmt, kc_chunk** out,
                          uint64_t* n_out) {
    if (!out || !n_out || k < 1 || (!dev_image && size)) return KC_ERR_ARG;
    if (hipDeviceSynchronize() != hipSuccess) return KC_ERR_HIP;  // the image's producers are done
    DeviceImg img{dev_image, size, {}};
    const int rc = plan_chunks_impl(img, size, k, chunk_size, fmt, out, n_out);
    if (rc == KC_OK && img.bad) {
        std::free(*out);
        *out = nullptr;
        *n_out = 0;
        return KC_ERR_HIP;
    }
    return rc;
}

uint64_t kc_table_size_reference(uint64_t at_least) {  // next_prime3mod4, functions_math.cpp:53-96
    if (at_least <= 2) return 2;
    uint64_t p = at_least % 2 == 0 ? at_least + 1 : at_least;
    for (;; p += 2) {
        bool prime = true;
        for (uint64_t d = 3; d * d <= p; d += 2)
            if (p % d == 0) { prime = false; break; }
        if (prime && p % 4 == 3) return p;
    }
}

int kc_xxh64(const uint64_t* values, const uint64_t* seeds, uint64_t n, uint64_t* out) {
    if (n && (!values || !seeds || !out)) return KC_ERR_ARG;
    if (n == 0) return KC_OK;
    uint64_t* d = nullptr;
    if (hipMalloc(&d, n * 3 * 8) != hipSuccess) return KC_ERR_NOMEM;
    hipError_t e = hipMemcpy(d, values, n * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d + n, seeds, n * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_xxh64(d, d + n, n, d + 2 * n, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, d + 2 * n, n * 8, hipMemcpyDeviceToHost);
    hipFree(d);
    return e == hipSuccess ? KC_OK : KC_ERR_HIP;
}

int kc_bloom_info(kc_ctx* c, uint64_t* n_words, uint64_t* bits, int* nh, int* nh_gate, int* layout) {
    if (!c) return KC_ERR_ARG;
    if (!c->d_bloom) return c->fail(KC_ERR_STATE, "no Bloom filter");
    if (n_words) *n_words = bloom_words(c);
    if (bits) *bits = c->bf_bits;
    if (nh) *nh = c->nh;
    if (nh_gate) *nh_gate = c->nh_gate;
    if (layout) *layout = c->bloom_blocked;
    return KC_OK;
}

int kc_bloom_read(kc_ctx* c, uint32_t* words, uint64_t n) {
    if (!c || (!words && n)) return KC_ERR_ARG;
    if (!c->d_bloom) return c->fail(KC_ERR_STATE, "no Bloom filter");
    if (n > bloom_words(c)) return c->fail(KC_ERR_ARG, "more words than the filter holds");
    int rc = kc_sync(c);
    if (rc) return rc;
    HIPCHK(c, hipMemcpy(words, c->d_bloom, n * 4, hipMemcpyDeviceToHost));
    return KC_OK;
}

int kc_bloom_write(kc_ctx* c, const uint32_t* words, uint64_t n) {
    if (!c || (!words && n)) return KC_ERR_ARG;
    if (!c->d_bloom) return c->fail(KC_ERR_STATE, "no Bloom filter");
    if (n > bloom_words(c)) return c->fail(KC_ERR_ARG, "more words than the filter holds");
    int rc = kc_sync(c);
    if (rc) return rc;
    HIPCHK(c, hipMemcpy(c->d_bloom, words, n * 4, hipMemcpyHostToDevice));
    c->bloom_fresh = false;
    return KC_OK;
}

// Work on stream s after everything the context staged from the host (its own stream).
static int after_host_work(kc_ctx* c, hipStream_t s) {
    int rc = flush_host(c);
    if (rc) return rc;
    if (s != c->stream) {
        HIPCHK(c, hipEventRecord(c->xev, c->stream));
        HIPCHK(c, hipStreamWaitEvent(s, c->xev, 0));
    }
    return KC_OK;
}

int kc_bloom_get_device(kc_ctx* c, uint32_t* dev_dst, uint64_t first_word, uint64_t n_words, void* sp) {
    if (!c || (!dev_dst && n_words)) return KC_ERR_ARG;
    if (!c->d_bloom) return c->fail(KC_ERR_STATE, "no Bloom filter");
    if (first_word > bloom_words(c) || n_words > bloom_words(c) - first_word)
        return c->fail(KC_ERR_ARG, "word range outside the filter");
    hipStream_t s = pick_stream(c, sp);
    int rc = after_host_work(c, s);
    if (rc) return rc;
    if (n_words) HIPCHK(c, hipMemcpyAsync(dev_dst, c->d_bloom + first_word, n_words * 4, hipMemcpyDeviceToDevice, s));
    return KC_OK;
}

int kc_bloom_merge_device(kc_ctx* c, const uint32_t* dev_parts, uint32_t nparts, uint64_t n_words, uint32_t* dev_out,
                          void* sp) {
    if (!c || nparts == 0 || (n_words && (!dev_parts || !dev_out))) return KC_ERR_ARG;
    if (!c->d_bloom) return c->fail(KC_ERR_STATE, "no Bloom filter");
    if (c->bloom_blocked && n_words % 16) return c->fail(KC_ERR_ARG, "the blocked filter merges whole 16-word blocks");
    HIPCHK(c, launch_bloom_merge(dev_parts, nparts, n_words, c->bloom_blocked, dev_out, pick_stream(c, sp)));
    return KC_OK;
}

// Distinct k-mers in filter 2 from its set bits (after the work queued on s): X of m bits set
// after n insertions of h positions each, X = m (1 - e^{-hn/m}).
static int estimate_filter2(kc_ctx* c, hipStream_t s, uint64_t* est) {
    unsigned long long* part_d = c->d_sum + CHECKSUM_SLOTS;  // the first CHECKSUM_SLOTS hold the reuse checksum
    HIPCHK(c, launch_bloom_popcount2(c->d_bloom, bloom_words(c), c->bloom_blocked, part_d, s));
    unsigned long long part[CHECKSUM_SLOTS];
    HIPCHK(c, hipMemcpyAsync(part, part_d, sizeof(part), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    double x = 0;
    for (auto v : part) x += (double)v;
    const double m = c->bloom_blocked ? 256.0 * (double)bloom_blocks(c->bf_bits) : (double)c->bf_bits;
    x = std::min(x, m - 1);
    *est = (uint64_t)std::llround(-(m / std::max(1, c->nh)) * std::log1p(-x / m));
    return KC_OK;
}

int kc_bloom_set_device(kc_ctx* c, const uint32_t* dev_src, uint64_t n_words, uint64_t* new_in_second, void* sp) {
    if (!c || !dev_src) return KC_ERR_ARG;
    if (!c->cfg.bf_enable || c->bloom_final) return c->fail(KC_ERR_STATE, "bloom pass not active");
    if (n_words != bloom_words(c)) return c->fail(KC_ERR_ARG, "n_words must be the filter's word count");
    hipStream_t s = pick_stream(c, sp);
    int rc = after_host_work(c, s);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(c->d_bloom, dev_src, n_words * 4, hipMemcpyDeviceToDevice, s));
    c->bloom_fresh = false;
    uint64_t est = 0;
    rc = estimate_filter2(c, s, &est);  // waits for the copy
    if (rc) return rc;
    // the pass-1 counter kc_bloom_finalize sizes the table from (main.cpp:454)
    HIPCHK(c, hipMemcpy(&c->d_ctr->new_in_second, &est, 8, hipMemcpyHostToDevice));
    if (new_in_second) *new_in_second = est;
    return KC_OK;
}

int kc_bloom_estimate(kc_ctx* c, uint64_t* distinct_in_second, void* sp) {
    if (!c || !distinct_in_second) return KC_ERR_ARG;
    if (!c->d_bloom) return c->fail(KC_ERR_STATE, "no Bloom filter");
    hipStream_t s = pick_stream(c, sp);
    int rc = after_host_work(c, s);
    if (rc) return rc;
    return estimate_filter2(c, s, distinct_in_second);
}

uint64_t kc_synth_bytes(uint64_t first_read, uint64_t n_reads, uint32_t read_len, uint32_t wrap) {
    kc_synth_params p{};
    p.read_len = read_len;
    p.wrap = wrap;
    return kcs_record_offset(&p, first_read + n_reads) - kcs_record_offset(&p, first_read);
}

int kc_synth_device(uint8_t* dst, uint64_t first_read, uint64_t n_reads, uint64_t seed, uint64_t genome_len,
                    uint32_t read_len, uint32_t wrap, double err_rate, double n_rate, void* s) {
    if (!dst || genome_len < read_len || read_len == 0) return KC_ERR_ARG;
    hipError_t e = launch_synth(dst, first_read, n_reads, seed, genome_len, read_len, wrap, err_rate, n_rate,
                                nullptr, (hipStream_t)s);
    return e == hipSuccess ? KC_OK : KC_ERR_HIP;
}

int kc_synth_skew_device(uint8_t* dst, uint64_t first_read, uint64_t n_reads, uint64_t seed, uint64_t genome_len,
                         uint32_t read_len, uint32_t wrap, double err_rate, double n_rate, const kc_synth_skew* skew,
                         void* s) {
    if (!dst || genome_len < read_len || read_len == 0) return KC_ERR_ARG;
    hipError_t e = launch_synth(dst, first_read, n_reads, seed, genome_len, read_len, wrap, err_rate, n_rate, skew,
                                (hipStream_t)s);
    return e == hipSuccess ? KC_OK : KC_ERR_HIP;
}

}  // extern "C"
