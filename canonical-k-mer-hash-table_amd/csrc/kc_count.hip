// kc_count.hip -- W-dispatch of the counting entry points (kc_internal.h launch_*): the
// kernels of every key width W = 1..15 live in their own translation unit
// (kc_count_w.hip -DKC_W=W, kernels in kc_count_impl.h).
#include "kc_internal.h"

namespace kc {

#define KC_DISPATCH_W(W_, CALL)                \
    switch (W_) {                              \
    case 1: return WOps<1>::CALL;              \
    case 2: return WOps<2>::CALL;              \
    case 3: return WOps<3>::CALL;              \
    case 4: return WOps<4>::CALL;              \
    case 5: return WOps<5>::CALL;              \
    case 6: return WOps<6>::CALL;              \
    case 7: return WOps<7>::CALL;              \
    case 8: return WOps<8>::CALL;              \
    case 9: return WOps<9>::CALL;              \
    case 10: return WOps<10>::CALL;            \
    case 11: return WOps<11>::CALL;            \
    case 12: return WOps<12>::CALL;            \
    case 13: return WOps<13>::CALL;            \
    case 14: return WOps<14>::CALL;            \
    case 15: return WOps<15>::CALL;            \
    default: return hipErrorInvalidValue;      \
    }

hipError_t launch_count(PackedView sym, uint64_t sym_bound, int k, int mode, TableView t, BloomView bf,
                        DevCounters* ctr, hipStream_t s) {
    KC_DISPATCH_W(t.W, count(sym, sym_bound, k, mode, t, bf, ctr, s));
}

hipError_t launch_count_partitioned(PackedView sym, uint64_t sym_bound, int k, int mode, TableView t, BloomView bf,
                                    DevCounters* ctr, PartBufs pb, int fresh, hipStream_t s, int phase) {
    (void)sym_bound;
    KC_DISPATCH_W(t.W, count_partitioned(sym, k, mode, t, bf, ctr, pb, fresh, s, phase));
}

// the blocked layout's filter regions: R divides the block count, <= 1024 blocks each
hipError_t launch_bloom_partitioned(PackedView sym, int k, int W, BloomView bf, TableView ft, TableView fg,
                                    DevCounters* ctr, PartBufs pb, int fresh, int keep, hipStream_t s, int phase) {
    if (!bf.blocked || ft.R == 0 || bf.nblocks % ft.R || bf.nblocks / ft.R > (uint64_t)BF_BLOCKS_PER_REGION) return hipErrorInvalidValue;
    // the fine bins refine the filter regions (both powers of two)
    if (keep && (fg.R < ft.R || fg.R % ft.R || (fg.R & (fg.R - 1)))) return hipErrorInvalidValue;
    KC_DISPATCH_W(W, bloom_partitioned(sym, k, bf, ft, fg, ctr, pb, fresh, keep, s, phase));
}

hipError_t launch_count_reuse(int W, TableView t, BloomView bf, DevCounters* ctr, PartBufs pb, int fresh, int level,
                              int gate, uint64_t windows, hipStream_t s) {
    if (!bf.blocked || pb.cap1 == 0 || t.F1 * pb.B2 == 0) return hipErrorInvalidValue;
    KC_DISPATCH_W(W, count_reuse(t, bf, ctr, pb, fresh, level, gate, windows, s));
}

hipError_t launch_bloom_records(int W, const uint64_t* rec, uint64_t n, BloomView bf, TableView ft, DevCounters* ctr,
                                PartBufs pb, int fresh, hipStream_t s) {
    if (!bf.blocked || ft.R == 0 || bf.nblocks % ft.R || bf.nblocks / ft.R > (uint64_t)BF_BLOCKS_PER_REGION)
        return hipErrorInvalidValue;
    KC_DISPATCH_W(W, bloom_records(rec, n, bf, ft, ctr, pb, fresh, s));
}

hipError_t launch_count_records(int W, const uint64_t* rec, uint64_t n, TableView t, BloomView bf, DevCounters* ctr,
                                PartBufs pb, int fresh, int gate, hipStream_t s) {
    if (gate && !bf.blocked) return hipErrorInvalidValue;
    KC_DISPATCH_W(W, count_records(rec, n, t, bf, ctr, pb, fresh, gate, s));
}

hipError_t launch_route(PackedView sym, int k, int W, DevCounters* ctr, PartBufs pb, uint32_t parts, uint64_t* out,
                        hipStream_t s) {
    KC_DISPATCH_W(W, route(sym, k, ctr, pb, parts, out, s));
}

hipError_t launch_insert_keys(const uint64_t* keys, uint64_t n, bool partitioned, TableView t, DevCounters* ctr,
                              PartBufs pb, int fresh, hipStream_t s) {
    KC_DISPATCH_W(t.W, insert_keys(keys, n, partitioned, t, ctr, pb, fresh, s));
}

hipError_t launch_route_table(TableView t, uint32_t parts, uint32_t* hist, uint64_t* off, uint64_t* bsum,
                              uint64_t* out, hipStream_t s, int hist_ready) {
    if (parts == 0 || parts > RT_MAX_PARTS) return hipErrorInvalidValue;
    KC_DISPATCH_W(t.W, route_table(t, parts, hist, off, bsum, out, s, hist_ready));
}

hipError_t launch_insert_counts(const uint64_t* rec, uint64_t n, bool partitioned, TableView t, DevCounters* ctr,
                                PartBufs pb, int fresh, hipStream_t s) {
    KC_DISPATCH_W(t.W, insert_counts(rec, n, partitioned, t, ctr, pb, fresh, s));
}

#define KC_DISPATCH_CW(W_, CALL)               \
    switch (W_) {                              \
    case 1: return CompactOps<1>::CALL;        \
    case 2: return CompactOps<2>::CALL;        \
    case 3: return CompactOps<3>::CALL;        \
    case 4: return CompactOps<4>::CALL;        \
    case 5: return CompactOps<5>::CALL;        \
    case 6: return CompactOps<6>::CALL;        \
    case 7: return CompactOps<7>::CALL;        \
    case 8: return CompactOps<8>::CALL;        \
    case 9: return CompactOps<9>::CALL;        \
    case 10: return CompactOps<10>::CALL;      \
    case 11: return CompactOps<11>::CALL;      \
    case 12: return CompactOps<12>::CALL;      \
    case 13: return CompactOps<13>::CALL;      \
    case 14: return CompactOps<14>::CALL;      \
    case 15: return CompactOps<15>::CALL;      \
    default: return hipErrorInvalidValue;      \
    }

hipError_t launch_compact_build(TableView t, CompactView c, int k, hipStream_t s) {
    KC_DISPATCH_CW(t.W, build(t, c, k, s));
}
hipError_t launch_compact_dump(int W, CompactView c, int k, uint64_t a, uint64_t* out, unsigned long long* cursor,
                               unsigned long long* stats, hipStream_t s) {
    KC_DISPATCH_CW(W, dump(c, k, a, out, cursor, stats, s));
}
hipError_t launch_compact_lookup(int W, CompactView c, int k, const uint64_t* keys, uint64_t n, uint32_t* counts,
                                 hipStream_t s) {
    KC_DISPATCH_CW(W, lookup(c, k, keys, n, counts, s));
}

hipError_t launch_hll(PackedView sym, int k, int W, DevCounters* ctr, uint32_t* regs, hipStream_t s) {
    KC_DISPATCH_W(W, hll(sym, k, ctr, regs, s));
}

hipError_t launch_dump(TableView t, int count_mode, uint64_t min_abundance, uint64_t* out, DevCounters* ctr,
                       hipStream_t s) {
    KC_DISPATCH_W(t.W, dump(t, count_mode, min_abundance, out, ctr, s));
}

hipError_t launch_text_bytes(TableView t, int count_mode, uint64_t a, int k, uint32_t* block_bytes, uint64_t* off,
                             uint64_t* bsum, hipStream_t s) {
    const uint64_t nblk = (t.nbuckets + TEXT_T - 1) / TEXT_T;
    if (nblk == 0 || nblk > 0x7FFFFFFFull) return hipErrorInvalidValue;
    KC_DISPATCH_W(t.W, text_bytes(t, count_mode, a, k, block_bytes, off, bsum, s));
}

hipError_t launch_text(TableView t, int count_mode, uint64_t a, int k, uint64_t blk0, uint64_t nblk,
                       const uint64_t* off, uint64_t base, uint8_t* out, size_t lds, hipStream_t s) {
    if (nblk == 0) return hipSuccess;
    if (nblk > 0x7FFFFFFFull || lds > 160 * 1024) return hipErrorInvalidValue;
    KC_DISPATCH_W(t.W, text(t, count_mode, a, k, blk0, nblk, off, base, out, lds, s));
}

hipError_t launch_text_digest(TableView t, int count_mode, uint64_t a, int k, unsigned long long* out, hipStream_t s) {
    if ((t.nbuckets + TEXT_T - 1) / TEXT_T > 0x7FFFFFFFull) return hipErrorInvalidValue;
    KC_DISPATCH_W(t.W, text_digest(t, count_mode, a, k, out, s));
}

hipError_t launch_check_runs(const uint64_t* rec, const uint64_t* gstart, uint32_t G, uint64_t maxn, TableView t,
                             unsigned long long* flag, hipStream_t s) {
    if (G == 0) return hipSuccess;
    KC_DISPATCH_W(t.W, check_runs(rec, gstart, G, maxn, t, flag, s));
}

hipError_t launch_insert_counts_runs(const uint64_t* rec, const uint64_t* gstart, uint32_t G, TableView t,
                                     DevCounters* ctr, uint32_t* m_len, uint64_t* m_start, int fresh, hipStream_t s) {
    if (G == 0 || G > 64) return hipErrorInvalidValue;
    KC_DISPATCH_W(t.W, insert_counts_runs(rec, gstart, G, t, ctr, m_len, m_start, fresh, s));
}

}  // namespace kc
