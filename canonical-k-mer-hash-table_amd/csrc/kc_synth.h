/*
 * kc_synth.h -- seeded synthetic read generator shared by the CPU tool
 * (tools/kc_gen.c) and the device generator in kc_device.hip, so that both emit
 * byte-identical FASTA for the same parameters (SURVEY.md 8d workload spec:
 * uniform ACGT genome of length G, N reads of length L starting uniformly in
 * [0, G-L], 50 % reverse-complemented, i.i.d. substitutions at rate e, optional
 * N-symbols at rate n; FASTA ">r<i>\n<seq>\n", sequence optionally wrapped).
 *
 * The generator is counter based (splitmix64 finalizer over (seed, stream,
 * index)) instead of a sequential xoshiro stream, so the device can produce any
 * read independently and in parallel.
 */
#ifndef KC_SYNTH_H
#define KC_SYNTH_H
#include <stdint.h>

#if defined(__HIPCC__)
#define KC_HD __host__ __device__ __forceinline__
#else
#define KC_HD static inline
#endif

typedef struct {
    uint64_t seed;
    uint64_t genome_len;   /* G */
    uint64_t n_reads;      /* N */
    uint32_t read_len;     /* L */
    uint32_t wrap;         /* 0 = single-line sequence, else columns per line */
    double err_rate;       /* substitution rate */
    double n_rate;         /* rate of 'N' symbols */
    /* skewed workloads (all 0 = the uniform SURVEY.md 8d generator): a fraction of the
     * reads are homopolymers (poly-A, or poly-T when reverse-complemented) or (CA)n
     * dinucleotide repeats, and the genome carries `repeat_copies` copies of one
     * `repeat_len`-base repeat evenly spaced over it */
    double homo_frac;
    double dinuc_frac;
    uint32_t repeat_len;
    uint32_t repeat_copies;
} kc_synth_params;

KC_HD uint64_t kcs_mix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}
KC_HD uint64_t kcs_rand(uint64_t seed, uint64_t stream, uint64_t i, uint64_t j) {
    return kcs_mix(kcs_mix(seed ^ (stream << 56) ^ (i * 0xd1342543de82ef95ULL)) + j);
}
KC_HD uint64_t kcs_mulhi(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}
/* genome base p: 32 bases per 64-bit random word; inside a copy of the repeat, the
 * repeat's base (its own random stream) */
KC_HD int kcs_genome_base(const kc_synth_params *g, uint64_t p) {
    if (g->repeat_copies && g->repeat_len) {
        const uint64_t spacing = g->genome_len / g->repeat_copies;
        const uint64_t off = spacing ? p % spacing : 0;
        if (spacing >= g->repeat_len && off < g->repeat_len && p / spacing < g->repeat_copies)
            return (int)((kcs_rand(g->seed, 6, off >> 5, 0) >> (2 * (off & 31))) & 3);
    }
    return (int)((kcs_rand(g->seed, 1, p >> 5, 0) >> (2 * (p & 31))) & 3);
}
KC_HD uint64_t kcs_thresh(double rate) {
    if (rate <= 0.0) return 0;
    if (rate >= 1.0) return ~0ULL;
    return (uint64_t)(rate * 18446744073709551616.0);
}
KC_HD uint64_t kcs_thresh(double rate);
/* read kind: 0 genome, 1 homopolymer, 2 (CA)n */
KC_HD int kcs_read_kind(const kc_synth_params *p, uint64_t i) {
    if (p->homo_frac <= 0.0 && p->dinuc_frac <= 0.0) return 0;
    const uint64_t u = kcs_rand(p->seed, 7, i, 0);
    if (u < kcs_thresh(p->homo_frac)) return 1;
    if (u - kcs_thresh(p->homo_frac) < kcs_thresh(p->dinuc_frac)) return 2;
    return 0;
}
/* base j (0..L-1) of read i, as 0..3 or 4 = 'N' */
KC_HD int kcs_read_base(const kc_synth_params *p, uint64_t i, uint32_t j, uint64_t start, int rc,
                        uint64_t e_th, uint64_t n_th) {
    const int kind = kcs_read_kind(p, i);
    int b;
    if (kind == 1) b = rc ? 3 : 0;                                     /* poly-A / poly-T */
    else if (kind == 2) b = ((j + (uint32_t)(start & 1)) & 1) ? 0 : 1;  /* CACA... / ACAC... */
    else b = rc ? 3 - kcs_genome_base(p, start + (p->read_len - 1 - j)) : kcs_genome_base(p, start + j);
    if (e_th && kcs_rand(p->seed, 3, i, j) < e_th) b = (b + 1 + (int)(kcs_rand(p->seed, 4, i, j) % 3)) & 3;
    if (n_th && kcs_rand(p->seed, 5, i, j) < n_th) b = 4;
    return b;
}
KC_HD uint64_t kcs_read_start(const kc_synth_params *p, uint64_t i) {
    return kcs_mulhi(kcs_rand(p->seed, 2, i, 0), p->genome_len - p->read_len + 1);
}
KC_HD int kcs_read_rc(const kc_synth_params *p, uint64_t i) { return (int)(kcs_rand(p->seed, 2, i, 1) & 1); }

KC_HD int kcs_digits(uint64_t v) {
    int d = 1;
    while (v >= 10) { v /= 10; d++; }
    return d;
}
/* bytes of the sequence part of one record incl. its line breaks */
KC_HD uint64_t kcs_seq_bytes(const kc_synth_params *p) {
    uint64_t L = p->read_len;
    uint64_t lines = p->wrap ? (L + p->wrap - 1) / p->wrap : 1;
    return L + lines;
}
/* byte offset of record i (">r<i>\n" header = 3 + digits(i) bytes) */
KC_HD uint64_t kcs_record_offset(const kc_synth_params *p, uint64_t i) {
    uint64_t off = i * (3 + kcs_seq_bytes(p));
    uint64_t lo = 0, pow10 = 1;
    for (int d = 1; d <= 20; d++) {
        uint64_t hi = pow10 * 10;            /* numbers with d digits: [pow10, hi) (0 has 1 digit) */
        uint64_t a = lo, b = hi < i ? hi : i; /* count of indices j < i with d digits */
        if (b > a) off += (b - a) * (uint64_t)d;
        if (hi >= i) break;
        lo = hi;
        pow10 = hi;
    }
    return off;
}
KC_HD uint64_t kcs_total_bytes(const kc_synth_params *p) { return kcs_record_offset(p, p->n_reads); }
#endif
