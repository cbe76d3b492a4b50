// kc_compact_impl.h -- Kaarme's compact representation as a post-count compaction (SURVEY.md
// 8f row 3), kernels for one key width W (instantiated by kc_compact_w.hip).
//
// The reference stores every k-mer as one 8-byte slot word (OneCharacterAndPointerKMerAtomic-
// Variable, kmer.hpp:103-149, accessors kmer.cpp:610-714): bit 0 occupied, 1 predecessor
// exists, 4 "self canonical during insertion", 5 "predecessor canonical during insertion",
// 8-9 right and 10-11 left character of the canonical k-mer, 12-25 the count (saturating at
// 16383), 26-63 the predecessor's slot -- or, for a chain start (bit 1 clear), its index in
// the secondary array of full keys.  A k-mer is read back by walking predecessors and
// collecting one character per hop (reconstruct_kmer_in_slot, kmer_hash_table.cpp:3848-4058).
// The reference links a k-mer to the k-mer before it in the read that inserted it, during
// insertion (process_kmer_MT, kmer_hash_table.cpp:2207-2567: a latency-bound chain walk per
// window).  Here the full-key table is counted first and then compacted:
//
//  * every k-mer gets an orientation o (the "read" it is written in): the strand on which its
//    minimizer (the odd-length canonical m-mer of smallest hash) reads forward.  Neighbouring
//    k-mers of one genome strand share their minimizer most of the time, so they get the
//    same strand and read as consecutive k-mers of one read;
//  * X's predecessor is a k-mer P of the table with P_read = c + X_read[0..k-2] whose own
//    orientation is that one (o_P == [P_read is canonical]), so every hop of a walk moves the
//    same way along the frame and adds one character: any k-mer is rebuilt in <= k - 2 hops
//    (or fewer, from a chain start's full key).  X may be its own predecessor (AAAA...);
//  * a k-mer without such a predecessor is a chain start: its key goes to the secondary array.
// Slot words use the reference's exact bit layout and flag semantics, so the reference's
// reconstruction walk (restated in k_creco / reco) rebuilds them; the compact table is an
// open-addressed array (linear probing from the table key's top bits), so a k-mer's count is
// found by probing and comparing reconstructed keys (left/right characters first, as the
// reference's quick_kmer_slot_check_sus, kmer_hash_table.cpp:2732-2761).
#pragma once
#include "kc_common.h"

namespace kc {

constexpr uint64_t CW_OCC = 1, CW_PRED = 2, CW_SELF = 16, CW_PREDC = 32;
constexpr int CW_RIGHT = 8, CW_LEFT = 10, CW_CNT = 12, CW_PTR = 26;
constexpr uint64_t CW_NONE = ~0ULL;  // src[] of an empty compact slot

template <int W>
DEV uint32_t key_char(const uint64_t (&K)[W], int k, int j) {  // character j (0 = leftmost)
    const int pos = 2 * (k - 1 - j);
    const int wi = W - 1 - (pos >> 6);
    uint64_t w = 0;
#pragma unroll
    for (int i = 0; i < W; i++)
        if (i == wi) w = K[i];
    return (uint32_t)(w >> (pos & 63)) & 3;
}
template <int W>
DEV void or_char(uint64_t (&K)[W], int k, int j, uint32_t c) {
    const int pos = 2 * (k - 1 - j);
    const int wi = W - 1 - (pos >> 6);
#pragma unroll
    for (int i = 0; i < W; i++)
        if (i == wi) K[i] |= (uint64_t)c << (pos & 63);
}
// P = c followed by the first k - 1 characters of X
template <int W>
DEV void prepend_char(const uint64_t (&X)[W], uint32_t c, const RollConst& rk, uint64_t (&P)[W]) {
#pragma unroll
    for (int i = W - 1; i >= 1; i--) P[i] = (X[i] >> 2) | (X[i - 1] << 62);
    P[0] = X[0] >> 2;
#pragma unroll
    for (int i = 0; i < W; i++)
        if (i == rk.rc_word) P[i] |= (uint64_t)c << rk.rc_bit;
}
template <int W>
DEV bool key_le(const uint64_t (&a)[W], const uint64_t (&b)[W]) {
#pragma unroll
    for (int i = 0; i < W; i++)
        if (a[i] != b[i]) return a[i] < b[i];
    return true;
}
template <int W>
DEV bool key_eq(const uint64_t (&a)[W], const uint64_t (&b)[W]) {
    bool eq = true;
#pragma unroll
    for (int i = 0; i < W; i++) eq &= a[i] == b[i];
    return eq;
}

// the minimizer's strand: true if the smallest-hash canonical m-mer (m odd: no palindromes)
// reads forward in the canonical k-mer K
template <int W>
DEV bool minimizer_forward(const uint64_t (&K)[W], int k, int m) {
    const uint64_t mask = (1ULL << (2 * m)) - 1;
    uint64_t fw = 0, rv = 0, best = ~0ULL;
    bool ori = true;
    for (int j = 0; j < k; j++) {
        const uint32_t c = key_char<W>(K, k, j);
        fw = ((fw << 2) | c) & mask;
        rv = (rv >> 2) | ((uint64_t)(3 - c) << (2 * (m - 1)));
        if (j >= m - 1) {
            const bool f = fw < rv;
            const uint64_t h = fmix64((f ? fw : rv) ^ 0x632BE59BD9B4E019ULL);
            if (h < best) {
                best = h;
                ori = f;
            }
        }
    }
    return ori;
}
inline int minimizer_len(int k) { return k >= 15 ? 15 : ((k & 1) ? k : k - 1); }
// One scan of K's m-mers gives everything k_clink needs without rescanning each candidate
// predecessor (k - m + 1 fmix64 per candidate: most of the link time at k = 127).
// A candidate P = c + X[0..k-2] (X = K as its read shows it) has the m-mers of X at positions
// 0..k-m-1 plus one new m-mer in front, so minimizer_forward(canonical(P)) follows from the
// minimum over that range of X (and the orientation of its first and last occurrence: the
// scan runs backwards on P's strand when P is not canonical) and the new m-mer's hash.  Hash
// ~0 is never chosen and ties go to the first in scan order, exactly as minimizer_forward.
struct MinRange {
    uint64_t h = ~0ULL;  // smallest hash (~0: none)
    bool first = true, last = true;  // forward flag of its first / last occurrence
    DEV void add(uint64_t hh, bool f) {
        if (hh < h) {
            h = hh;
            first = last = f;
        } else if (hh == h && hh != ~0ULL) {
            last = f;
        }
    }
};
struct MinScan {
    bool ox;                // minimizer_forward(K)
    MinRange lo, hi;        // K's m-mers at positions 0..k-m-1 and 1..k-m (K's strand)
};
template <int W>
DEV MinScan minimizer_scan(const uint64_t (&K)[W], int k, int m) {
    const uint64_t mask = (1ULL << (2 * m)) - 1;
    uint64_t fw = 0, rv = 0, best = ~0ULL;
    MinScan r;
    r.ox = true;
    for (int j = 0; j < k; j++) {
        const uint32_t c = key_char<W>(K, k, j);
        fw = ((fw << 2) | c) & mask;
        rv = (rv >> 2) | ((uint64_t)(3 - c) << (2 * (m - 1)));
        if (j >= m - 1) {
            const int pos = j - (m - 1);
            const bool f = fw < rv;
            const uint64_t h = fmix64((f ? fw : rv) ^ 0x632BE59BD9B4E019ULL);
            if (h < best) {
                best = h;
                r.ox = f;
            }
            if (pos < k - m) r.lo.add(h, f);
            if (pos >= 1) r.hi.add(h, f);
        }
    }
    return r;
}
// minimizer_forward(canonical(P)) == pc for P = c + X[0..k-2], pc = [P is canonical]:
// xr = the m-mers of X at positions 0..k-m-1 on X's strand, X0 = X's first m - 1 characters
DEV bool pred_reads_forward(const MinRange& xr, uint64_t x0, uint32_t c, int m, bool pc) {
    const uint64_t mask = (1ULL << (2 * m)) - 1;
    const uint64_t fw = (((uint64_t)c << (2 * (m - 1))) | x0) & mask;
    uint64_t rv = 0;
    for (int i = 0; i < m; i++) rv = (rv << 2) | (3 - ((fw >> (2 * i)) & 3));
    const bool f0 = fw < rv;
    const uint64_t h0 = fmix64((f0 ? fw : rv) ^ 0x632BE59BD9B4E019ULL);
    bool ori;
    if (pc) {  // scan on P's strand: the new m-mer comes first
        ori = (h0 != ~0ULL && h0 <= xr.h) ? f0 : xr.h != ~0ULL ? xr.first : true;
    } else {   // scan on the other strand: X's m-mers first (last occurrence first), flags flip
        ori = (xr.h != ~0ULL && xr.h <= h0) ? !xr.last : h0 != ~0ULL ? !f0 : true;
    }
    return ori == pc;
}

DEV uint64_t cslot_of(uint64_t t0, uint64_t nslots) { return __umul64hi(t0, nslots); }

// k_cplace: every occupied slot of the full-key table claims a compact slot (count in place)
template <int W>
__global__ __launch_bounds__(256) void k_cplace(TableView tv, CompactView cv) {
    constexpr int S = BUCKET_WORDS / (W + 1);
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= tv.nbuckets * S) return;
    const uint64_t* b = tv.buckets + (g / S) * BUCKET_WORDS;
    const int s = (int)(g % S);
    const uint64_t t0 = b[s * W];
    if (t0 == EMPTY) return;
    const uint64_t c = b[S * W + s] & CNT_MASK;
    const uint64_t word = CW_OCC | ((c < 16383 ? c : 16383) << CW_CNT);
    uint64_t p = cslot_of(t0, cv.nslots);
    while (atomicCAS(reinterpret_cast<unsigned long long*>(cv.words + p), 0ULL, (unsigned long long)word) != 0ULL)
        p = p + 1 == cv.nslots ? 0 : p + 1;
    cv.src[p] = g;
    cv.inv[g] = p;
}

// compact slot holding table key tk, or CW_NONE (build): the key is looked up in the
// full-key table, whose probe sequence (the key's region, buckets from its start bucket,
// kc_common.h) ends at the first bucket with a free slot, so a missing predecessor costs one
// or two 128-byte bucket reads instead of a compact-array probe run at load 0.8 (each probe
// comparing a random bucket's key); the found slot maps to its compact slot through inv.
template <int W>
DEV uint64_t cfind_built(const TableView& tv, const CompactView& cv, const uint64_t (&tk)[W]) {
    constexpr int S = BUCKET_WORDS / (W + 1);
    const uint64_t region = region_of(tk[0], tv.R);
    uint32_t b = bucket_in_region(tk[0], tv.R);
    for (int probe = 0; probe < BPR; probe++) {
        const uint64_t bucket = region * BPR + b;
        const uint64_t* bk = tv.buckets + bucket * BUCKET_WORDS;
        bool free = false;
#pragma unroll
        for (int sl = 0; sl < S; sl++) {
            const uint64_t w0 = bk[sl * W];
            free |= w0 == EMPTY;
            if (w0 != tk[0]) continue;
            bool eq = true;
#pragma unroll
            for (int i = 1; i < W; i++) eq &= bk[sl * W + i] == tk[i];
            if (eq) return cv.inv[bucket * S + sl];
        }
        if (free) return CW_NONE;
        b = (b + 1) & (BPR - 1);
    }
    return CW_NONE;
}

// k_clink: orientation, predecessor and flags of every compact slot; chain starts -> secondary
template <int W>
__global__ __launch_bounds__(256) void k_clink(TableView tv, CompactView cv, int k, int m) {
    constexpr int S = BUCKET_WORDS / (W + 1);
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t g = p < cv.nslots ? cv.src[p] : CW_NONE;
    const RollConst rk = make_roll<W>(k, 0, 0);
    uint64_t K[W], word = 0, pred = CW_NONE;
    bool start = false;
    if (g != CW_NONE) {
        uint64_t t[W];
        const uint64_t* key = tv.buckets + (g / S) * BUCKET_WORDS + (g % S) * W;
#pragma unroll
        for (int i = 0; i < W; i++) t[i] = key[i];
        from_tkey<W>(t, K);
        uint64_t rcK[W], X[W];
        revcomp<W>(K, rk, rcK);
        const MinScan ms = minimizer_scan<W>(K, k, m);
        const bool ox = ms.ox;
#pragma unroll
        for (int i = 0; i < W; i++) X[i] = ox ? K[i] : rcK[i];  // X as its read shows it
        // X's m-mers at positions 0..k-m-1 on X's strand: K's first k-m (ox) or, reversed and
        // flipped, K's last k-m
        MinRange xr = ms.lo;
        if (!ox) {
            xr = ms.hi;
            const bool f = xr.first;
            xr.first = !xr.last;
            xr.last = !f;
        }
        uint64_t x0 = 0;  // X's first m - 1 characters
        for (int j = 0; j < m - 1; j++) x0 = (x0 << 2) | key_char<W>(X, k, j);
        bool op = false;
        for (uint32_t c = 0; c < 4 && pred == CW_NONE; c++) {
            uint64_t P[W], rP[W], KP[W], tp[W];
            prepend_char<W>(X, c, rk, P);
            revcomp<W>(P, rk, rP);
            const bool pc = key_le<W>(P, rP);  // P as read is canonical
            canonical<W>(P, rP, KP);
            if (!pred_reads_forward(xr, x0, c, m, pc)) continue;  // P reads the other way
            to_tkey<W>(KP, tp);
            pred = cfind_built<W>(tv, cv, tp);
            op = pc;
        }
        word = cv.words[p] & (CW_OCC | (16383ULL << CW_CNT));
        word |= (uint64_t)key_char<W>(K, k, k - 1) << CW_RIGHT | (uint64_t)key_char<W>(K, k, 0) << CW_LEFT;
        if (ox) word |= CW_SELF;
        if (pred != CW_NONE) {
            word |= CW_PRED | (op ? CW_PREDC : 0) | (pred << CW_PTR);
        } else {
            start = true;
        }
    }
    // chain starts: one atomic per wave for their secondary-array indices
    const uint64_t ballot = __ballot(start);
    const int lane = threadIdx.x & 63;
    unsigned long long base = 0;
    if (ballot) {
        if (lane == __ffsll((long long)ballot) - 1) base = atomicAdd(cv.n_second, (unsigned long long)__popcll(ballot));
        base = __shfl(base, __ffsll((long long)ballot) - 1, 64);
    }
    if (start) {
        const uint64_t idx = base + __popcll(ballot & ((1ULL << lane) - 1));
#pragma unroll
        for (int i = 0; i < W; i++) cv.second[idx * W + i] = K[i];
        word |= idx << CW_PTR;
    }
    if (g != CW_NONE) cv.words[p] = word;
}

// reconstruct_kmer_in_slot (kmer_hash_table.cpp:3848-4058) on the compact words: the k-mer
// of slot p into K; hops = predecessors visited; false if the walk does not end in 4k hops
template <int W>
DEV bool reco(const CompactView& cv, uint64_t p, int k, uint64_t (&K)[W], uint32_t& hops) {
#pragma unroll
    for (int i = 0; i < W; i++) K[i] = 0;
    int L = 0, R = k - 1, Lc = 0, Rc = k - 1;
    bool pir = false;
    hops = 0;
    uint64_t w = cv.words[p];
    while (w & CW_PRED) {
        const uint32_t lch = (uint32_t)(w >> CW_LEFT) & 3, rch = (uint32_t)(w >> CW_RIGHT) & 3;
        if (L == Lc) {
            or_char<W>(K, k, L, pir ? 3 - rch : lch);
            if (++L > R) return true;
        }
        if (R == Rc) {
            or_char<W>(K, k, R, pir ? 3 - lch : rch);
            if (--R < L) return true;
        }
        const bool self = (w & CW_SELF) != 0, predc = (w & CW_PREDC) != 0;
        if (self != pir) { Lc--; Rc--; } else { Lc++; Rc++; }  // the eight cases of :3925-3998
        if (self != predc) pir = !pir;
        w = cv.words[w >> CW_PTR];
        if (++hops > 4 * (uint32_t)k) return false;
    }
    // chain start: the remaining characters from its full key (get_secondary_array_char)
    const uint64_t* sk = cv.second + (w >> CW_PTR) * W;
    uint64_t S[W];
#pragma unroll
    for (int i = 0; i < W; i++) S[i] = sk[i];
    const int Ls = L - Lc;
    for (int a = L, b = pir ? k - Ls - 1 : Ls; a <= R; a++, b += pir ? -1 : 1) {
        if (b < 0 || b >= k) return false;
        const uint32_t ch = key_char<W>(S, k, b);
        or_char<W>(K, k, a, pir ? 3 - ch : ch);
    }
    return true;
}

// k_creco: every occupied compact slot with T(c) >= a -> record {W key words, T(c)};
// stats[0] += hops, stats[1] = max hops, stats[2] += walks that did not end
template <int W>
__global__ __launch_bounds__(256) void k_creco(CompactView cv, int k, uint64_t a, uint64_t* __restrict__ out,
                                               unsigned long long* __restrict__ cursor,
                                               unsigned long long* __restrict__ stats) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t w = p < cv.nslots ? cv.words[p] : 0;
    const uint64_t cnt = (w >> CW_CNT) & 16383;
    const bool emit = (w & CW_OCC) && cnt >= a;
    uint64_t K[W];
    uint32_t hops = 0;
    bool ok = true;
    if (emit) ok = reco<W>(cv, p, k, K, hops);
    const uint64_t ballot = __ballot(emit);
    const int lane = threadIdx.x & 63;
    unsigned long long base = 0;
    if (ballot && out) {
        if (lane == __ffsll((long long)ballot) - 1) base = atomicAdd(cursor, (unsigned long long)__popcll(ballot));
        base = __shfl(base, __ffsll((long long)ballot) - 1, 64);
    }
    if (emit && out) {
        uint64_t* o = out + (base + __popcll(ballot & ((1ULL << lane) - 1))) * (W + 1);
#pragma unroll
        for (int i = 0; i < W; i++) o[i] = K[i];
        o[W] = cnt;
    }
    unsigned long long h = hops, mx = hops, bad = ok ? 0 : 1, n = emit ? 1 : 0;
    for (int o = 32; o >= 1; o >>= 1) {
        h += __shfl_xor(h, o, 64);
        bad += __shfl_xor(bad, o, 64);
        n += __shfl_xor(n, o, 64);
        const unsigned long long y = __shfl_xor(mx, o, 64);
        mx = y > mx ? y : mx;
    }
    if (lane == 0) {
        if (h) atomicAdd(stats + 0, h);
        if (mx) atomicMax(stats + 1, mx);
        if (bad) atomicAdd(stats + 2, bad);
        if (n && !out) atomicAdd(cursor, n);
    }
}

// k_clookup: T(c) of canonical keys (W words each) from the compact words alone (0 = absent)
template <int W>
__global__ __launch_bounds__(256) void k_clookup(CompactView cv, int k, const uint64_t* __restrict__ keys, uint64_t n,
                                                 uint32_t* __restrict__ counts) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t Q[W], tq[W];
#pragma unroll
    for (int j = 0; j < W; j++) Q[j] = keys[i * W + j];
    to_tkey<W>(Q, tq);
    const uint32_t ql = key_char<W>(Q, k, 0), qr = key_char<W>(Q, k, k - 1);
    uint64_t p = cslot_of(tq[0], cv.nslots);
    uint32_t res = 0;
    for (uint64_t probes = 0; probes < cv.nslots; probes++) {
        const uint64_t w = cv.words[p];
        if (!(w & CW_OCC)) break;
        if (((w >> CW_LEFT) & 3) == ql && ((w >> CW_RIGHT) & 3) == qr) {
            uint64_t K[W];
            uint32_t hops;
            if (reco<W>(cv, p, k, K, hops) && key_eq<W>(K, Q)) {
                res = (uint32_t)((w >> CW_CNT) & 16383);
                break;
            }
        }
        p = p + 1 == cv.nslots ? 0 : p + 1;
    }
    counts[i] = res;
}

template <int W>
hipError_t CompactOps<W>::build(TableView t, CompactView c, int k, hipStream_t s) {
    const uint64_t n = t.nbuckets * (BUCKET_WORDS / (W + 1));
    if (n) hipLaunchKernelGGL(k_cplace<W>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, t, c);
    hipLaunchKernelGGL(k_clink<W>, dim3((unsigned)((c.nslots + 255) / 256)), dim3(256), 0, s, t, c, k,
                       minimizer_len(k));
    return hipGetLastError();
}
template <int W>
hipError_t CompactOps<W>::dump(CompactView c, int k, uint64_t a, uint64_t* out, unsigned long long* cursor,
                               unsigned long long* stats, hipStream_t s) {
    hipLaunchKernelGGL(k_creco<W>, dim3((unsigned)((c.nslots + 255) / 256)), dim3(256), 0, s, c, k, a, out, cursor,
                       stats);
    return hipGetLastError();
}
template <int W>
hipError_t CompactOps<W>::lookup(CompactView c, int k, const uint64_t* keys, uint64_t n, uint32_t* counts,
                                 hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_clookup<W>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, k, keys, n, counts);
    return hipGetLastError();
}

}  // namespace kc
