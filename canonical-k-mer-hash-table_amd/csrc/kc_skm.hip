// kc_skm.hip -- super-k-mer routing for the multi-GPU exchange.
//
// The owner of a canonical k-mer is a hash of its canonical minimizer: the smallest value of
// h(canonical m-mer) over the k - m + 1 m-mers of the k-mer, mixed again (skm_owner).  A k-mer and its reverse complement
// hold the same canonical m-mers, so every occurrence of a canonical k-mer goes to one owner
// (exact counts, as SURVEY 8e's hash-prefix owner), and consecutive windows of a read share their
// minimizer -- and so their owner -- for ~(k - m + 2) / 2 windows on average.  A maximal run of r
// consecutive valid windows with one owner (a super-k-mer) travels as its k - 1 + r symbols,
// 2-bit packed, instead of r keys: ~1 byte per window at k = 51 against the 24-byte {key, count}
// records of the pre-aggregated exchange (sharded.py), whose per-rank coverage at C4 / 8 ranks
// gives ~0.4 distinct k-mers per window.
//
// Output: per owner, a symbol stream in the tokenizer's packed format (kc_internal.h PackedView:
// pk[w] holds symbols 32w .. 32w + 31 at bits 62 - 2j, bk[w] their break flags at bit 31 - j).
// Every super-k-mer is one break symbol followed by its k - 1 + r symbols, so the owner counts
// the stream with the ordinary levels (kc_count_packed_device) and no window spans two
// super-k-mers.  Each workgroup tile reserves a whole-word range per owner (one atomicAdd per
// owner and tile, order free: counting is order-independent) and pads its tail with breaks.
#include "kc_common.h"

namespace kc {

constexpr int SKM_T = 512;             // threads per workgroup
constexpr int SKM_RUN = 8;             // window ends per thread
constexpr int SKM_TP = SKM_T * SKM_RUN;  // window ends per tile
constexpr int SKM_MAXW = MAX_K;        // most m-mers per window (k - m + 1 <= k)
constexpr int SKM_STAGE = 1024;        // staged output words per tile (32 768 symbols)
constexpr int SKM_IN = (SKM_TP + SKM_MAXW) / 32 + 4;  // staged input words per tile
constexpr uint32_t SKM_BROKEN = 0xFFFFFFFFu;

DEV uint32_t fmix32(uint32_t h) {  // murmur3's finalizer (a bijection)
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h;
}
// h(canonical m-mer) in 32 bits, never SKM_BROKEN: two 32-bit multiplies (a 64-bit fmix64 took
// six of the kernel's per-position multiplies; m <= 16 m-mers fit the low word, so distinct m-mers
// keep distinct hashes)
DEV uint32_t mmer_hash(uint64_t canon) {
    const uint32_t h = fmix32((uint32_t)canon ^ (uint32_t)(canon >> 32) * SKM_FOLD ^ SKM_SEED32);
    return h == SKM_BROKEN ? SKM_BROKEN - 1 : h;
}

// the owner of a minimizer value: the minimum of w uniform hashes is small, so it is mixed again
// (murmur3's fmix32) before the multiply-shift onto the owners
DEV uint32_t skm_owner(uint32_t minh, uint32_t nshards) {
    return (uint32_t)(((uint64_t)fmix32(minh ^ 0x9E3779B9u) * nshards) >> 32);
}

// 32 symbols starting at symbol s of the tile's staged input words (word wlo of the stream at
// stage index 0; s >= 32 wlo)
DEV uint64_t load32_at(const uint64_t* __restrict__ st, int64_t wlo, int64_t s) {
    const int64_t w = (s >> 5) - wlo;  // (arithmetic shift: floor)
    const int o = (int)(s & 31);
    const uint64_t a = st[w], b = st[w + 1];
    return o ? (a << (2 * o)) | (b >> (64 - 2 * o)) : a;
}

// Write `len` symbols starting at input symbol `src` into the output at symbol `dst` (a break
// symbol precedes them at dst - 1, set by the caller), OR-ing words into an LDS stage or, for
// a tile whose output does not fit the stage, its global range.
DEV void put_symbols(uint64_t* __restrict__ opk, const uint64_t* __restrict__ st, int64_t wlo, int64_t src,
                     uint64_t dst, uint64_t len) {
    const uint64_t w0 = dst >> 5, w1 = (dst + len - 1) >> 5;
    for (uint64_t w = w0; w <= w1; w++) {
        // input symbol of output slot 32w (before src for the first word: those slots are masked off,
        // and the stage holds a word before src's)
        const int64_t s0 = max(src + (int64_t)(w * 32) - (int64_t)dst, (int64_t)(wlo * 32));
        uint64_t v = load32_at(st, wlo, s0);
        if (src + (int64_t)(w * 32) - (int64_t)dst < s0) v >>= 2 * (s0 - (src + (int64_t)(w * 32) - (int64_t)dst));
        // keep the output slots [dst, dst + len) of this word
        const uint64_t lo = w * 32 < dst ? dst - w * 32 : 0;
        const uint64_t hi = (w + 1) * 32 > dst + len ? dst + len - w * 32 : 32;
        uint64_t m = (hi - lo == 32) ? ~0ULL : (((1ULL << (2 * (hi - lo))) - 1) << (2 * (32 - hi)));
        v &= m;
        atomicOr(reinterpret_cast<unsigned long long*>(opk + w), (unsigned long long)v);
    }
}

// One workgroup per tile of SKM_TP window ends (grid-stride over tiles).
//   out_pk / out_bk: nshards regions of cap words each; cursor[o]: words used in region o (grows
//   past cap on overflow: the caller's retry size); wins[o]: windows routed to o; ovf: set when a
//   region overflowed (nothing of that tile is written for that owner).
__global__ __launch_bounds__(SKM_T) void k_skm_route(PackedView sv, const DevCounters* __restrict__ ctr, int k, int m,
                                                     uint32_t nshards, uint64_t* __restrict__ out_pk,
                                                     uint32_t* __restrict__ out_bk, uint64_t cap,
                                                     unsigned long long* __restrict__ cursor,
                                                     unsigned long long* __restrict__ wins,
                                                     unsigned long long* __restrict__ ovf) {
    // s_u: the m-mer hashes (steps 1-2), then each window end's run length and offset (steps 3-5)
    constexpr int NU = (SKM_TP + SKM_MAXW) > (SKM_TP * 3 / 2) ? (SKM_TP + SKM_MAXW) : (SKM_TP * 3 / 2);
    __shared__ uint32_t s_u[NU];
    uint32_t* s_h = s_u;
    uint32_t* s_off = s_u;                                          // [SKM_TP]
    uint16_t* s_run = reinterpret_cast<uint16_t*>(s_u + SKM_TP);   // [SKM_TP]
    __shared__ uint64_t s_ipk[SKM_IN + 1];  // the tile's input words (symbols t0 - k + 1 .. t1)
    __shared__ uint32_t s_ibk[SKM_IN + 1];
    __shared__ uint8_t s_ow[SKM_TP];
    __shared__ uint64_t s_pk[SKM_STAGE];
    __shared__ uint32_t s_bk[SKM_STAGE];
    __shared__ uint32_t s_cnt[SKM_MAX_SHARDS], s_win[SKM_MAX_SHARDS], s_lbase[SKM_MAX_SHARDS + 1];
    __shared__ unsigned long long s_gbase[SKM_MAX_SHARDS];
    __shared__ int s_direct;
    __shared__ uint16_t s_starts[SKM_TP];  // the tile's super-k-mer starts (step 3), in any order
    __shared__ uint32_t s_nstart, s_wtot[SKM_T / 64];
    __shared__ uint32_t s_wmin[SKM_T / 64];
    const int tid = threadIdx.x;
    const uint64_t M = ctr->stream_len;
    const int w = k - m + 1;  // m-mers per window
    const uint64_t mmask = m >= 32 ? ~0ULL : (1ULL << (2 * m)) - 1;
    const int rsh = 64 - 2 * m;
    const uint64_t ntiles = (M + SKM_TP - 1) / SKM_TP;
    const int j0 = tid * SKM_RUN;  // first window end of this thread (tile-relative)
    // (step 1's layout of the m-mer hashes: row i % SKM_RUN, column i / SKM_RUN; the row pitch is 8
    // words past a multiple of the 64 banks, so a wave's 8 x 8 writes of step 1 hit 64 banks too)
    constexpr int HP = ((SKM_TP + SKM_MAXW) / SKM_RUN + 1 + 63) / 64 * 64 + 8;
    static_assert(SKM_RUN == 8 && HP * SKM_RUN <= NU, "the interleaved hashes fit s_u");
    auto hix = [](int i) { return (i & (SKM_RUN - 1)) * HP + (i >> 3); };
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t t0 = tile * SKM_TP, t1 = min(t0 + SKM_TP, M);
        const int tlen = (int)(t1 - t0);
        // 0. the tile's input words into LDS: symbols t0 - k + 1 .. t1 (+ one word: 32-symbol loads)
        const int64_t wlo = ((int64_t)t0 - (k - 1)) >> 5;
        const int nin = (int)((int64_t)((t1 - 1) >> 5) + 2 - wlo);
        for (int i = tid; i < nin; i += SKM_T) {
            const int64_t gw = wlo + i;
            const bool in = gw >= 0 && (uint64_t)gw <= ((M - 1) >> 5) + 1;
            s_ipk[i] = in ? sv.pk[gw] : 0;
            s_ibk[i] = in ? sv.bk[gw] : 0xFFFFFFFFu;
        }
        if (tid < (int)nshards) {
            s_cnt[tid] = 0;
            s_win[tid] = 0;
        }
        __syncthreads();
        // 1. the hashes of the m-mers ending at t0 - w + 1 .. t1 - 1 (broken: a break symbol inside,
        //    or the m-mer starts before the stream).  Thread t rolls the SKM_RUN consecutive m-mers
        //    8t .. 8t + 7 (one extraction, then a symbol each); the rest (the w - 1 past the tile's
        //    SKM_TP) one by one.  m-mer i sits at s_h[hix(i)]: the SKM_RUN m-mers of a thread in SKM_RUN
        //    rows, so that the lanes of a wave touch consecutive words here and in step 2 (a thread's
        //    m-mers side by side put the lanes 8 words apart: 8-way LDS bank conflicts, 20 % of the
        //    kernel's cycles)
        const int nh = tlen + w - 1;
        auto mmer_at = [&](int i) {  // one m-mer from scratch
            const int64_t q = (int64_t)t0 - (w - 1) + i;  // last symbol of the m-mer
            const int64_t a = q - m + 1;
            uint32_t h = SKM_BROKEN;
            if (a >= 0) {
                const int64_t wa = (a >> 5) - wlo, wq = (q >> 5) - wlo;
                uint32_t br = s_ibk[wa] & (0xFFFFFFFFu >> (a & 31));
                if (wq != wa) br = br ? br : (s_ibk[wq] & (0xFFFFFFFFu << (31 - (q & 31))));
                else br &= 0xFFFFFFFFu << (31 - (q & 31));
                if (!br) {
                    const uint64_t x = (load32_at(s_ipk, wlo, a) >> rsh) & mmask;  // m symbols, oldest first
                    const uint64_t rc = (rev2(~x) >> rsh) & mmask;
                    h = mmer_hash(x < rc ? x : rc);
                }
            }
            return h;
        };
        {
            const int i0 = j0;  // this thread's first m-mer
            if (i0 < nh) {
                const int64_t q0 = (int64_t)t0 - (w - 1) + i0, a0 = q0 - m + 1;
                // consecutive non-break symbols ending at q0 (capped at m; none before the stream)
                int since = 0;
                if (q0 >= 0) {
                    const int64_t wq = (q0 >> 5) - wlo;
                    const uint32_t mq = s_ibk[wq] & (0xFFFFFFFFu << (31 - (q0 & 31)));
                    if (mq) {
                        since = (int)(q0 & 31) - (31 - __builtin_ctz(mq));
                    } else {
                        const uint32_t mp = wq > 0 ? s_ibk[wq - 1] : 0xFFFFFFFFu;
                        since = (int)(q0 & 31) + 1 + (mp ? 31 - (31 - __builtin_ctz(mp)) : 32);
                    }
                    since = (int)min((int64_t)min(since, m), q0 + 1);
                }
                uint64_t x = 0, rc = 0;
                if (a0 >= -32) {  // (a stage word exists before the stream's first)
                    x = (load32_at(s_ipk, wlo, a0) >> rsh) & mmask;
                    rc = (rev2(~x) >> rsh) & mmask;
                }
                s_h[hix(i0)] = since >= m ? mmer_hash(x < rc ? x : rc) : SKM_BROKEN;
                // the next SKM_RUN - 1 symbols and their break bits
                const int64_t q1 = q0 + 1;
                const uint64_t ins = load32_at(s_ipk, wlo, q1);
                const int64_t wb = (q1 >> 5) - wlo;
                const int ob = (int)(q1 & 31);
                const uint32_t inb = ob ? (s_ibk[wb] << ob) | (s_ibk[wb + 1] >> (32 - ob)) : s_ibk[wb];
                const int rcs = 2 * (m - 1);
#pragma unroll
                for (int j = 1; j < SKM_RUN; j++) {
                    const uint32_t c = (uint32_t)(ins >> (62 - 2 * (j - 1))) & 3;
                    const bool brk = (inb >> (31 - (j - 1))) & 1;
                    since = brk ? 0 : min(since + 1, m);
                    x = ((x << 2) | c) & mmask;
                    rc = (rc >> 2) | ((uint64_t)(3 - c) << rcs);
                    if (i0 + j < nh) s_h[hix(i0 + j)] = since >= m ? mmer_hash(x < rc ? x : rc) : SKM_BROKEN;
                }
            }
            for (int i = SKM_TP + tid; i < nh; i += SKM_T) s_h[hix(i)] = mmer_at(i);
        }
        __syncthreads();
        // 2. per window end: valid (no broken m-mer among its w) and the minimizer -> owner.  Window j
        //    covers s_h[j0 + j .. j0 + j + w - 1]: for w >= SKM_RUN the part common to the thread's
        //    SKM_RUN windows [j0 + SKM_RUN - 1, j0 + w - 1], a left part [j0 + j, j0 + SKM_RUN - 2]
        //    (suffixes) and a right part [j0 + w, j0 + w + j - 1] (prefixes): w + 2 SKM_RUN reads
        {
            auto hv = [&](int i) { return i < nh ? s_h[hix(i)] : SKM_BROKEN; };
            uint32_t mn[SKM_RUN], mx[SKM_RUN];
            if (w >= SKM_RUN) {
                uint32_t cmn = SKM_BROKEN, cmx = 0;
                for (int i = j0 + SKM_RUN - 1; i <= j0 + w - 1; i++) {
                    const uint32_t h = hv(i);
                    cmn = min(cmn, h);
                    cmx = max(cmx, h);
                }
                uint32_t ln = cmn, lx = cmx;
#pragma unroll
                for (int j = SKM_RUN - 1; j >= 0; j--) {
                    if (j < SKM_RUN - 1) {
                        const uint32_t h = hv(j0 + j);
                        ln = min(ln, h);
                        lx = max(lx, h);
                    }
                    mn[j] = ln;
                    mx[j] = lx;
                }
                uint32_t rn = SKM_BROKEN, rx = 0;
#pragma unroll
                for (int j = 0; j < SKM_RUN; j++) {
                    if (j > 0) {
                        const uint32_t h = hv(j0 + w + j - 1);
                        rn = min(rn, h);
                        rx = max(rx, h);
                    }
                    mn[j] = min(mn[j], rn);
                    mx[j] = max(mx[j], rx);
                }
            } else {
#pragma unroll
                for (int j = 0; j < SKM_RUN; j++) {
                    uint32_t a = SKM_BROKEN, b = 0;
                    for (int i = j0 + j; i < j0 + j + w; i++) {
                        const uint32_t h = hv(i);
                        a = min(a, h);
                        b = max(b, h);
                    }
                    mn[j] = a;
                    mx[j] = b;
                }
            }
            __syncthreads();  // (s_h is read no more: its space holds the runs below)
#pragma unroll
            for (int j = 0; j < SKM_RUN; j++) {
                const bool valid = j0 + j < tlen && mx[j] != SKM_BROKEN;
                s_ow[j0 + j] = valid ? (uint8_t)skm_owner(mn[j], nshards) : 0xFF;
            }
        }
        __syncthreads();
        // 3. super-k-mer starts: run length, symbols (a break + k - 1 + r), offset in the owner's range.
        //    A run ends at the next boundary (a position whose owner differs from its predecessor's, or
        //    the tile's end): the thread's first boundary, then a suffix minimum of those over the
        //    threads (wave shuffles + one LDS pass over the waves), so every run length is O(1)
        {
            uint32_t bmask = 0;  // bit j: window end j0 + j is a boundary
            uint8_t prev = j0 == 0 ? 0xFE : (j0 - 1 < tlen ? s_ow[j0 - 1] : 0xFF);
#pragma unroll
            for (int j = 0; j < SKM_RUN; j++) {
                const uint8_t o = j0 + j < tlen ? s_ow[j0 + j] : 0xFF;
                if (o != prev || j0 + j >= tlen) bmask |= 1u << j;
                prev = o;
            }
            uint32_t fb = bmask ? (uint32_t)(j0 + __builtin_ctz(bmask)) : (uint32_t)SKM_TP;
            // suffix minimum over the threads after this one: within the wave by shuffles, then the waves'
            const int lane = tid & 63, wv = tid >> 6;
            uint32_t sfx = fb;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_down(sfx, d, 64);
                if (lane + d < 64) sfx = min(sfx, o);
            }
            if (lane == 0) s_wmin[wv] = sfx;
            __syncthreads();
            uint32_t after = __shfl_down(sfx, 1, 64);  // the suffix minimum from the next thread
            if (lane == 63) after = SKM_TP;
            for (int v = wv + 1; v < SKM_T / 64; v++) after = min(after, s_wmin[v]);
            uint32_t smask = 0;  // bit j: a super-k-mer starts at window end j0 + j
#pragma unroll
            for (int j = 0; j < SKM_RUN; j++) {
                const int p = j0 + j;
                uint32_t r = 0;
                if ((bmask >> j) & 1 && p < tlen && s_ow[p] != 0xFF) {
                    const uint32_t later = bmask & ~((2u << j) - 1);  // boundaries after p in this thread
                    const uint32_t e = min(later ? (uint32_t)(j0 + __builtin_ctz(later)) : after, (uint32_t)tlen);
                    r = e - (uint32_t)p;
                    smask |= 1u << j;
                }
                s_run[p] = (uint16_t)r;
            }
            // the tile's list of starts: a block scan of the threads' counts (no per-start atomics
            // under a branch: each of a thread's 8 slots had waited for its own LDS atomic)
            const uint32_t cnt = (uint32_t)__builtin_popcount(smask), incl = wave_incl_sum(cnt);
            if (lane == 63) s_wtot[wv] = incl;
            __syncthreads();
            uint32_t at = incl - cnt;
            for (int v = 0; v < wv; v++) at += s_wtot[v];
            if (tid == SKM_T - 1) s_nstart = at + cnt;
            for (uint32_t mk = smask; mk; mk &= mk - 1) s_starts[at++] = (uint16_t)(j0 + __builtin_ctz(mk));
        }
        __syncthreads();
        // each start's offset in its owner's range (order free: counting does not depend on it)
        for (uint32_t i = tid; i < s_nstart; i += SKM_T) {
            const int p = s_starts[i];
            const uint32_t o = s_ow[p], r = s_run[p];
            s_off[p] = atomicAdd(&s_cnt[o], (uint32_t)k + r);
            atomicAdd(&s_win[o], r);
        }
        __syncthreads();
        // 4. whole-word ranges per owner: global (one atomicAdd each) and the LDS stage layout
        if (tid == 0) {
            uint32_t acc = 0;
            for (uint32_t o = 0; o < nshards; o++) {
                s_lbase[o] = acc;
                acc += (s_cnt[o] + 31) / 32;
            }
            s_lbase[nshards] = acc;
            s_direct = acc > SKM_STAGE;
        }
        if (tid < (int)nshards) {
            const uint32_t nw = (s_cnt[tid] + 31) / 32;
            unsigned long long g = ~0ULL;
            if (nw) {
                g = atomicAdd(&cursor[tid], (unsigned long long)nw);
                atomicAdd(&wins[tid], (unsigned long long)s_win[tid]);
                if (g + nw > cap) {
                    atomicOr(ovf, 1ULL);
                    g = ~0ULL;
                }
            }
            s_gbase[tid] = g;
        }
        __syncthreads();
        const bool direct = s_direct != 0;
        const uint32_t tot = s_lbase[nshards];
        if (!direct) {
            for (uint32_t i = tid; i < tot; i += SKM_T) {
                s_pk[i] = 0;
                s_bk[i] = 0;
            }
        } else {
            // (more than the stage holds: this tile ORs straight into its global ranges, zeroed first)
            for (uint32_t o = 0; o < nshards; o++) {
                const unsigned long long g = s_gbase[o];
                if (g == ~0ULL) continue;
                const uint32_t nw = (s_cnt[o] + 31) / 32;
                for (uint32_t i = tid; i < nw; i += SKM_T) {
                    out_pk[o * cap + g + i] = 0;
                    out_bk[o * cap + g + i] = 0;
                }
            }
            __threadfence();
        }
        __syncthreads();
        // 5. the super-k-mers' symbols and separators, one start per thread from the tile's list (a
        //    thread's own 8 window ends held ~0.4 starts: each of the 8 slots ran the symbol copy for
        //    the few lanes with a start there); the tail of each owner's range: breaks
        const uint32_t nst = s_nstart;
#pragma unroll 1
        for (uint32_t i = tid; i < nst; i += SKM_T) {
            const int p = s_starts[i];
            const uint32_t r = s_run[p];
            const uint32_t o = s_ow[p], off = s_off[p];
            const uint64_t d = (uint64_t)off + 1;  // after the separator
            const int64_t src = (int64_t)(t0 + p) - (k - 1);
            const uint64_t len = (uint64_t)k - 1 + r;
            if (!direct) {
                const uint64_t base = (uint64_t)s_lbase[o] * 32;
                atomicOr(&s_bk[(base + off) >> 5], 0x80000000u >> ((base + off) & 31));
                put_symbols(s_pk, s_ipk, wlo, src, base + d, len);
            } else if (s_gbase[o] != ~0ULL) {
                const uint64_t base = (s_gbase[o] + o * cap) * 32;
                atomicOr(&out_bk[(base + off) >> 5], 0x80000000u >> ((base + off) & 31));
                put_symbols(out_pk, s_ipk, wlo, src, base + d, len);
            }
        }
        if (tid < (int)nshards && s_cnt[tid] % 32) {
            const uint32_t used = s_cnt[tid] % 32;  // the last word's padding symbols are breaks
            const uint32_t pad = 0xFFFFFFFFu >> used;
            const uint32_t lw = (s_cnt[tid] + 31) / 32 - 1;
            if (!direct)
                atomicOr(&s_bk[s_lbase[tid] + lw], pad);
            else if (s_gbase[tid] != ~0ULL)
                atomicOr(&out_bk[tid * cap + s_gbase[tid] + lw], pad);
        }
        __syncthreads();
        // 6. staged tiles: copy each owner's words to its global range
        if (!direct) {
            for (uint32_t o = 0; o < nshards; o++) {
                const unsigned long long g = s_gbase[o];
                const uint32_t lb = s_lbase[o], nw = s_lbase[o + 1] - lb;
                if (g == ~0ULL) continue;
                for (uint32_t i = tid; i < nw; i += SKM_T) {
                    out_pk[o * cap + g + i] = s_pk[lb + i];
                    out_bk[o * cap + g + i] = s_bk[lb + i];
                }
            }
        }
        __syncthreads();
    }
}

hipError_t launch_skm_route(PackedView sv, const DevCounters* ctr, uint64_t sym_bound, int k, int m, uint32_t nshards,
                            uint64_t* out_pk, uint32_t* out_bk, uint64_t cap, unsigned long long* cursor,
                            unsigned long long* wins, unsigned long long* ovf, hipStream_t s) {
    if (nshards == 0 || nshards > SKM_MAX_SHARDS || m < 1 || m > 32 || m > k) return hipErrorInvalidValue;
    const uint64_t tiles = (sym_bound + SKM_TP - 1) / SKM_TP;
    const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(tiles, 256 * 16));
    hipLaunchKernelGGL(k_skm_route, dim3(grid), dim3(SKM_T), 0, s, sv, ctr, k, m, nshards, out_pk, out_bk, cap, cursor,
                       wins, ovf);
    return hipGetLastError();
}

}  // namespace kc
