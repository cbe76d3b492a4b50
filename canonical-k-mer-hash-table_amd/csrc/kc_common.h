// kc_common.h -- device helpers shared by the tokenizer (kc_tokenize.hip) and the
// counting kernels (kc_count.hip): symbol codes, hashing, wave scans, the 2-bit
// canonical window roller, XXH64 and the table geometry.
#pragma once
#include "kc_internal.h"

namespace kc {

#define DEV __device__ __forceinline__

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

// ---- table keys -------------------------------------------------------------------
// The table stores the canonical key through a bijection ("tkey"), word 0 a strong mix of the
// whole key and never 0 (0 marks an empty slot):
//   W = 1:  t0 = tmix(key0 ^ MIX_C)
//   W >= 2: t0 = tmix(x), x = key[W-1] ^ g(key[0..W-2]); t1 = key0; t[i] = key[i-1] (i >= 2)
//           (x = 0 is stored as tmix(TK_ZERO) with TK_FLAG set in t1)
// tmix(x) = y ^ (y >> 32) with y = x * TMUL (odd, so both steps are bijections): one 64-bit
// multiply per window.  The top bits of y (regions, buckets, coarse bins) depend on every bit
// of x; the low half (shard owner) is folded with the high half.  For W >= 2 the last key word
// (the newest 32 characters) goes through the mix and word 1 keeps key word 0, which holds only
// the 2k - 64(W-1) <= 62 oldest-character bits: a level record of a two-word key needs t0's
// bits below its bin plus those bits (kc_count_impl.h Rec12).  The hash is computed once per
// window, every later level is a bit field of tkey word 0, and k_dump inverts the mix.
// W = 1: key0 < 2^62 and MIX_C has bit 63 set, so the tmix argument is never 0 and neither is
// t0 (tmix(x) = 0 only for x = 0).
constexpr uint64_t MIX_C = 0x9E3779B97F4A7C15ULL;  // bit 63 set
constexpr uint64_t M62 = (1ULL << 62) - 1;
constexpr uint64_t TMUL = 0x9E3779B97F4A7C15ULL;      // odd
constexpr uint64_t TMUL_INV = 0xF1DE83E19937733DULL;  // TMUL * TMUL_INV = 1 (mod 2^64)
constexpr uint64_t TK_ZERO = 0x6A09E667F3BCC909ULL;   // the stand-in of a zero mix argument
constexpr uint64_t TK_FLAG = 1ULL << 62;              // t1: the mix argument was 0

DEV uint64_t tmix(uint64_t x) {
    const uint64_t y = x * TMUL;
    return y ^ (y >> 32);
}
DEV uint64_t tmix_inv(uint64_t t) {
    return (t ^ (t >> 32)) * TMUL_INV;  // y ^ (y >> 32) is an involution
}
// hash of key words 0 .. W-2 (W >= 2)
template <int W>
DEV uint64_t side_hash(const uint64_t (&w)[W]) {
    uint64_t g = 0;
#pragma unroll
    for (int i = 0; i + 1 < W; i++) g = fmix64(g ^ w[i] ^ (0x243f6a8885a308d3ULL * (i + 1)));
    return g;
}
template <int W>
DEV void to_tkey(const uint64_t (&key)[W], uint64_t (&t)[W]) {
    if constexpr (W == 1) {
        t[0] = tmix(key[0] ^ MIX_C);
    } else {
        const uint64_t x = key[W - 1] ^ side_hash<W>(key);
        t[0] = tmix(x ? x : TK_ZERO);
        t[1] = key[0] | (x ? 0 : TK_FLAG);
#pragma unroll
        for (int i = 2; i < W; i++) t[i] = key[i - 1];
    }
}
template <int W>
DEV void from_tkey(const uint64_t (&t)[W], uint64_t (&key)[W]) {
    if constexpr (W == 1) {
        key[0] = tmix_inv(t[0]) ^ MIX_C;
    } else {
        key[0] = t[1] & ~TK_FLAG;
#pragma unroll
        for (int i = 2; i < W; i++) key[i - 1] = t[i];
        key[W - 1] = ((t[1] & TK_FLAG) ? 0 : tmix_inv(t[0])) ^ side_hash<W>(key);
    }
}

// ---- table geometry -------------------------------------------------------------
// Region r = floor(x * R / 2^32) with x = the top 32 bits of tkey word 0 (multiply-shift,
// so R need not be a power of two); the start bucket is the top BPR_BITS of the
// fraction (x * R mod 2^32), uniform and independent of r.  Linear probing wraps inside
// the region, so a region is an independent table that fits in LDS.  For R = F1 * F2
// (F2 a power of two) the level-1 bin of a key is r >> log2 F2 and its level-2 bin
// r & (F2 - 1).  The shard owner (multi-GPU) uses the low 32 bits, independent of both.
// R < 2^32 (kc_api.cpp alloc_table): one 32 x 32 -> 64-bit product gives the region (high
// half) and the fraction (low half)
DEV uint64_t region_of(uint64_t t0, uint64_t R) { return __umulhi((uint32_t)(t0 >> 32), (uint32_t)R); }
DEV uint32_t bucket_in_region(uint64_t t0, uint64_t R) {
    return ((uint32_t)(t0 >> 32) * (uint32_t)R) >> (32 - BPR_BITS);
}
DEV uint32_t owner_of(uint64_t t0, uint32_t parts) { return (uint32_t)(((t0 & 0xFFFFFFFFULL) * parts) >> 32); }

// wave-level inclusive scans (64 lanes).  The sum runs on DPP lane moves (no LDS
// round trips): row_shr 1/2/4/8 inside each 16-lane row, then row_bcast:15 (rows 1 and 3
// add the last lane of the row below) and row_bcast:31 (rows 2 and 3 add lane 31); lanes
// with no source lane add 0.
DEV uint32_t wave_incl_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
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

// ---- XXH64 of one 8-byte value (xxhash.h:3368-3509 / doc/xxhash_spec.md:191-334) ----
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

// ---- XXH64 of `len` bytes at any alignment (the same spec, every input length): the per-line
// hash of the output digest (kc_output_digest; oracle/kc_digest.c hashes the reference's text) ----
DEV uint64_t rd_le(const uint8_t* p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v |= (uint64_t)p[i] << (8 * i);
    return v;
}
DEV uint64_t xxh64_bytes(const uint8_t* p, uint32_t len, uint64_t seed) {
    const uint64_t P1 = 0x9E3779B185EBCA87ULL, P2 = 0xC2B2AE3D27D4EB4FULL, P3 = 0x165667B19E3779F9ULL,
                   P4 = 0x85EBCA77C2B2AE63ULL, P5 = 0x27D4EB2F165667C5ULL;
    auto round = [&](uint64_t acc, uint64_t in) { return rotl64(acc + in * P2, 31) * P1; };
    const uint8_t* end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        do {
            v1 = round(v1, rd_le(p, 8));
            v2 = round(v2, rd_le(p + 8, 8));
            v3 = round(v3, rd_le(p + 16, 8));
            v4 = round(v4, rd_le(p + 24, 8));
            p += 32;
        } while (p + 32 <= end);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = (h ^ round(0, v1)) * P1 + P4;
        h = (h ^ round(0, v2)) * P1 + P4;
        h = (h ^ round(0, v3)) * P1 + P4;
        h = (h ^ round(0, v4)) * P1 + P4;
    } else {
        h = seed + P5;
    }
    h += len;
    for (; p + 8 <= end; p += 8) h = rotl64(h ^ round(0, rd_le(p, 8)), 27) * P1 + P4;
    if (p + 4 <= end) {
        h = rotl64(h ^ (rd_le(p, 4) * P1), 23) * P2 + P3;
        p += 4;
    }
    for (; p < end; p++) h = rotl64(h ^ ((uint64_t)*p * P5), 11) * P1;
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

DEV uint64_t atomic_load_agent(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
DEV void atomic_store_agent(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- canonical window roller ------------------------------------------------------
// KMerFactoryCanonical2BC::push_new_integer (kmer_factory.cpp:172-239): forward word
// grows at the low end, reverse complement at the top; canonical = min as a 2k-bit
// integer.  With a Bloom filter the Rabin-Karp pair mod 2^54 of RollingHasherDual
// (hash_functions.cpp:102-192) is rolled alongside and root = min(F, B).
constexpr uint64_t M54 = (1ULL << 54) - 1;
constexpr uint64_t INV5_54 = 0xCCCCCCCCCCCCDULL;  // 5 * INV5_54 == 1 (mod 2^54)

struct RollConst {
    int k;
    int top;          // bits of the k-mer held by word 0
    int rc_word;      // word and bit of the oldest character (2k-2)
    int rc_bit;
    uint64_t topmask;
    uint64_t pow5_k, pow5_km1;
};

template <int W>
DEV RollConst make_roll(int k, uint64_t pk, uint64_t pkm1) {
    RollConst r;
    r.k = k;
    r.top = 2 * k - 64 * (W - 1);
    r.topmask = r.top >= 64 ? ~0ULL : ((1ULL << r.top) - 1);
    r.rc_word = W - 1 - (2 * k - 2) / 64;
    r.rc_bit = (2 * k - 2) % 64;
    r.pow5_k = pk;
    r.pow5_km1 = pkm1;
    return r;
}

// symbol p of the packed stream: 0..3, or 4 for a break
DEV uint32_t sym_at(const PackedView& sv, uint64_t p) {
    if ((sv.bk[p >> 5] >> (31 - (p & 31))) & 1) return SYM_BREAK;
    return (uint32_t)(sv.pk[p >> 5] >> (62 - 2 * (p & 31))) & 3;
}

// Rolls symbols [pstart, pend) and calls f(fwd, rc, root) for every complete window whose
// last symbol is at p >= p0.  ROOT: also roll the mod-2^54 pair (Bloom modes).
template <int W, bool ROOT, class F>
DEV void roll_run(const PackedView& sv, uint64_t pstart, uint64_t p0, uint64_t pend, const RollConst& rk, F&& f) {
    uint64_t fwd[W], rc[W];
#pragma unroll
    for (int i = 0; i < W; i++) { fwd[i] = 0; rc[i] = 0; }
    int fill = 0;
    uint64_t Fh = 0, Bh = 0, p5 = 1;
    for (uint64_t p = pstart; p < pend; p++) {
        const uint32_t c = sym_at(sv, p);
        if (c > 3) {
            fill = 0;
#pragma unroll
            for (int i = 0; i < W; i++) { fwd[i] = 0; rc[i] = 0; }
            if constexpr (ROOT) { Fh = 0; Bh = 0; p5 = 1; }
            continue;
        }
        if constexpr (ROOT) {
            if (fill < rk.k) {
                Fh = (Fh * 5 + c) & M54;
                Bh = (Bh + (uint64_t)(3 - c) * p5) & M54;
                p5 = (p5 * 5) & M54;
            } else {
                uint64_t out = 0;
#pragma unroll
                for (int i = 0; i < W; i++)
                    if (i == rk.rc_word) out = (fwd[i] >> rk.rc_bit) & 3;
                Fh = (Fh * 5 + c - rk.pow5_k * out) & M54;
                Bh = (((Bh - (3 - out)) & M54) * INV5_54 + (uint64_t)(3 - c) * rk.pow5_km1) & M54;
            }
        }
#pragma unroll
        for (int i = 0; i < W - 1; i++) fwd[i] = (fwd[i] << 2) | (fwd[i + 1] >> 62);
        fwd[W - 1] = (fwd[W - 1] << 2) | c;
        fwd[0] &= rk.topmask;
#pragma unroll
        for (int i = W - 1; i >= 1; i--) rc[i] = (rc[i] >> 2) | (rc[i - 1] << 62);
        rc[0] >>= 2;
#pragma unroll
        for (int i = 0; i < W; i++)
            if (i == rk.rc_word) rc[i] |= (uint64_t)(3 - c) << rk.rc_bit;
        if (fill < rk.k) fill++;
        if (fill == rk.k && p >= p0) f(fwd, rc, Fh < Bh ? Fh : Bh);
    }
}

// ---- direct window extraction (no rolling) -----------------------------------------
// The window ending at symbol `last` is the contiguous bit range of the big-endian packed
// stream: W funnel shifts of adjacent words; valid iff no break bit in [last-k+1, last].
template <int W>
DEV bool extract_window(const PackedView& sv, uint64_t last, const RollConst& rk, uint64_t (&fwd)[W]) {
    if (last + 1 < (uint64_t)rk.k) return false;
    const uint64_t a = last + 1 - rk.k;
    const uint64_t wa = a >> 5, wl = last >> 5;
    for (uint64_t w = wa; w <= wl; w++) {
        uint32_t m = sv.bk[w];
        if (w == wa) m &= 0xFFFFFFFFu >> (a & 31);
        if (w == wl) m &= 0xFFFFFFFFu << (31 - (last & 31));
        if (m) return false;
    }
    const int s = 2 * ((int)(last & 31) + 1);  // 2..64
    uint64_t lo = sv.pk[wl];
#pragma unroll
    for (int i = 0; i < W; i++) {
        const uint64_t hi = wl >= (uint64_t)(i + 1) ? sv.pk[wl - i - 1] : 0;
        fwd[W - 1 - i] = s == 64 ? lo : ((hi << s) | (lo >> (64 - s)));
        lo = hi;
    }
    fwd[0] &= rk.topmask;
    return true;
}

DEV uint64_t rev2(uint64_t x) {  // reverse the order of the 32 two-bit groups
    x = ((x >> 2) & 0x3333333333333333ULL) | ((x & 0x3333333333333333ULL) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0FULL) | ((x & 0x0F0F0F0F0F0F0F0FULL) << 4);
    return __builtin_bswap64(x);
}

// reverse complement of the k-mer held in the low 2k bits of the W-word integer
template <int W>
DEV void revcomp(const uint64_t (&f)[W], const RollConst& rk, uint64_t (&r)[W]) {
    uint64_t t[W];
#pragma unroll
    for (int i = 0; i < W; i++) t[i] = rev2(~f[W - 1 - i]);
    const int sh = 64 * W - 2 * rk.k;  // 2..64
    const int q = sh >> 6, b = sh & 63;
#pragma unroll
    for (int i = 0; i < W; i++) {
        const int src = i - q;
        uint64_t v = 0;
        if (src >= 0) v = b ? (t[src] >> b) : t[src];
        if (b && src - 1 >= 0) v |= t[src - 1] << (64 - b);
        r[i] = v;
    }
    r[0] &= rk.topmask;
}

template <int W>
DEV void canonical(const uint64_t (&fwd)[W], const uint64_t (&rc)[W], uint64_t (&key)[W]) {
    bool fwd_le = true;
#pragma unroll
    for (int i = W - 1; i >= 0; i--)
        if (fwd[i] != rc[i]) fwd_le = fwd[i] < rc[i];
#pragma unroll
    for (int i = 0; i < W; i++) key[i] = fwd_le ? fwd[i] : rc[i];
}


// Word sources of run_windows: the packed stream in HBM, or a workgroup's LDS stage of the
// words [wb, wb + n) it covers (k_p1 loads the next tile's words while it scatters this one)
struct PkGlobal {
    const PackedView& sv;
    DEV uint64_t pk(uint64_t w) const { return sv.pk[w]; }
    DEV uint32_t bk(uint64_t w) const { return sv.bk[w]; }
};
struct PkStage {
    const uint64_t* p;
    const uint32_t* b;
    int64_t wb;
    DEV uint64_t pk(uint64_t w) const { return p[(int64_t)w - wb]; }
    DEV uint32_t bk(uint64_t w) const { return b[(int64_t)w - wb]; }
};

// Table keys of the RUNW consecutive windows ending at r0 .. r0+RUNW-1: the state of
// the window ending at r0-1 is extracted in O(1) (funnel shifts + the position of the
// last break), then RUNW unrolled rolling steps (kmer_factory.cpp:172-239) produce the
// rest, so every slot index is static.  ok[j] is false for windows that contain a
// break or end at or beyond t1.  Reads words (r0 - k) / 32 - 1 .. r0 / 32 + 1 of sv.
template <int W, int RUNW, class G>
DEV void run_windows(const PackedView& sv, uint64_t r0, uint64_t t1, const RollConst& rk, G&& emit);
template <int W, int RUNW, class Src, class G>
DEV void run_windows_src(const Src& sv, uint64_t r0, uint64_t t1, const RollConst& rk, G&& emit) {
    static_assert(RUNW <= 32, "run must fit two packed words");
    const int k = rk.k;
    uint64_t fwd[W], rc[W];
    int since;  // consecutive non-break symbols ending at r0-1, capped at k
    {
        // symbols [r0-k, r0-1]: words wl-W..wl of the packed stream
        const int64_t last = (int64_t)r0 - 1;
        if (last < 0) {
#pragma unroll
            for (int i = 0; i < W; i++) fwd[i] = 0;
            since = 0;
        } else {
            const uint64_t wl = (uint64_t)last >> 5;
            const int s = 2 * ((int)(last & 31) + 1);
            uint64_t lo = sv.pk(wl);
#pragma unroll
            for (int i = 0; i < W; i++) {
                const uint64_t hi = wl >= (uint64_t)(i + 1) ? sv.pk(wl - i - 1) : 0;
                fwd[W - 1 - i] = s == 64 ? lo : ((hi << s) | (lo >> (64 - s)));
                lo = hi;
            }
            fwd[0] &= rk.topmask;
            // last break at or before `last`, looking back at most k symbols
            const int64_t first = last - k + 1;
            since = k;
            const int64_t wfirst = first < 0 ? 0 : (first >> 5);
            for (int64_t w = (int64_t)wl; w >= wfirst; w--) {
                uint32_t m = sv.bk((uint64_t)w);
                if (w == (int64_t)wl) m &= 0xFFFFFFFFu << (31 - (last & 31));
                if (m) {
                    const int64_t q = (w << 5) + (31 - __builtin_ctz(m));  // highest-index break in word w
                    since = (int)min((int64_t)k, last - q);
                    break;
                }
            }
            if (first < 0 && since > last + 1) since = (int)(last + 1);  // the stream starts at 0
        }
        revcomp<W>(fwd, rk, rc);
    }
    const uint64_t wa = r0 >> 5;
    const uint64_t pa = sv.pk(wa), pb = sv.pk(wa + 1);
    const uint32_t ba = sv.bk(wa), bb = sv.bk(wa + 1);
    const int o0 = (int)(r0 & 31);
    // the run's RUNW incoming symbols and break bits, funnel-shifted into one register each, so
    // every step reads them at a constant position
    const uint64_t ins = o0 ? (pa << (2 * o0)) | (pb >> (64 - 2 * o0)) : pa;  // symbol j at bits 63-2j:62-2j
    const uint32_t inb = o0 ? (ba << o0) | (bb >> (32 - o0)) : ba;            // break j at bit 31-j
    if constexpr (W == 1) {
        const uint64_t top = rk.topmask;
        const int rcb = rk.rc_bit;
        uint64_t f = fwd[0], r = rc[0];
#pragma unroll
        for (int j = 0; j < RUNW; j++) {
            const uint32_t c = (uint32_t)(ins >> (62 - 2 * j)) & 3;
            const bool br = (inb >> (31 - j)) & 1;
            since = br ? 0 : min(since + 1, k);
            f = ((f << 2) | c) & top;
            r = (r >> 2) | ((uint64_t)(3 - c) << rcb);
            const uint64_t fo[1] = {f}, ro[1] = {r};
            emit(j, r0 + j < t1 && since >= k, fo, ro);
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < RUNW; j++) {
        const uint32_t c = (uint32_t)(ins >> (62 - 2 * j)) & 3;
        const bool br = (inb >> (31 - j)) & 1;
        since = br ? 0 : min(since + 1, k);
#pragma unroll
        for (int i = 0; i < W - 1; i++) fwd[i] = (fwd[i] << 2) | (fwd[i + 1] >> 62);
        fwd[W - 1] = (fwd[W - 1] << 2) | c;
        fwd[0] &= rk.topmask;
#pragma unroll
        for (int i = W - 1; i >= 1; i--) rc[i] = (rc[i] >> 2) | (rc[i - 1] << 62);
        rc[0] >>= 2;
#pragma unroll
        for (int i = 0; i < W; i++)
            if (i == rk.rc_word) rc[i] |= (uint64_t)(3 - c) << rk.rc_bit;
        emit(j, r0 + j < t1 && since >= k, fwd, rc);
    }
}

template <int W, int RUNW, class G>
DEV void run_windows(const PackedView& sv, uint64_t r0, uint64_t t1, const RollConst& rk, G&& emit) {
    run_windows_src<W, RUNW>(PkGlobal{sv}, r0, t1, rk, emit);
}

}  // namespace kc
