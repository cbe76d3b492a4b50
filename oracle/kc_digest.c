/*
 * kc_digest -- order-independent digest of Kaarme's output (TEST INFRASTRUCTURE ONLY: a
 * checker for tests/ and tests/golden/make_fullsize.py, never linked or run by the product;
 * see kc_oracle_core.h).
 *
 * Digest of a set of output lines "<CANONICAL_KMER> <T(c)>\n" (the result contract, SURVEY.md
 * 8a A18; the writer kmer_hash_table.cpp:4318-4524): {lines, sum of T(c), sum mod 2^64 and XOR of
 * XXH64(line bytes incl. '\n', seed 0)}.  Any line order gives the same digest and the digests
 * of disjoint line sets add up, so it is what the engine's kc_output_digest computes per table
 * (per owner of a sharded job) and what a job too large to sort is checked by.
 *
 *   kc_digest lines [FILE|-]
 *       digest of a Kaarme output file (e.g. the reference's, oracle/_ref/kaarme -o FIFO).
 *   kc_digest count INPUT K [-m M] [-a A] [-c CHUNK] [-p PARTS] [-j THREADS]
 *       the restatement's count of INPUT (kc_oracle_core.h: the reference chunking, tokenizer,
 *       canonical keys and count transform -- the same functions kc_oracle count uses) and the
 *       digest of its output, without holding every k-mer at once: the canonical k-mers are split
 *       into PARTS partitions by a hash of the key, every partition is counted by its own scan of
 *       the whole input (THREADS partitions at a time), and the partitions' digests are added.
 *       No Bloom filter: with -b and a >= 2 the reference's output equals the unfiltered one
 *       (SURVEY.md 8a A18), so a Bloom case's digest is the count's at its -a.
 * Prints one JSON object: lines, count_sum, hash_sum / hash_xor (16 hex digits), and for count
 * windows and distinct.
 */
#include "kc_oracle_core.h"

#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

/* XXH64 of any length (xxhash.h:3368-3509 XXH64_endian_align / doc/xxhash_spec.md:191-334) */
static inline uint64_t rd64(const unsigned char *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v; /* little-endian host (x86-64), as the spec reads lanes */
}
static inline uint64_t rd32(const unsigned char *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
static inline uint64_t xround(uint64_t acc, uint64_t in) {
    return kco_rotl64(acc + in * KCO_P64_2, 31) * KCO_P64_1;
}
static uint64_t xxh64(const unsigned char *p, size_t len, uint64_t seed) {
    const unsigned char *end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + KCO_P64_1 + KCO_P64_2, v2 = seed + KCO_P64_2, v3 = seed, v4 = seed - KCO_P64_1;
        do {
            v1 = xround(v1, rd64(p));
            v2 = xround(v2, rd64(p + 8));
            v3 = xround(v3, rd64(p + 16));
            v4 = xround(v4, rd64(p + 24));
            p += 32;
        } while (p + 32 <= end);
        h = kco_rotl64(v1, 1) + kco_rotl64(v2, 7) + kco_rotl64(v3, 12) + kco_rotl64(v4, 18);
        h = (h ^ xround(0, v1)) * KCO_P64_1 + KCO_P64_4;
        h = (h ^ xround(0, v2)) * KCO_P64_1 + KCO_P64_4;
        h = (h ^ xround(0, v3)) * KCO_P64_1 + KCO_P64_4;
        h = (h ^ xround(0, v4)) * KCO_P64_1 + KCO_P64_4;
    } else {
        h = seed + KCO_P64_5;
    }
    h += (uint64_t)len;
    for (; p + 8 <= end; p += 8) h = kco_rotl64(h ^ xround(0, rd64(p)), 27) * KCO_P64_1 + KCO_P64_4;
    if (p + 4 <= end) {
        h = kco_rotl64(h ^ (rd32(p) * KCO_P64_1), 23) * KCO_P64_2 + KCO_P64_3;
        p += 4;
    }
    for (; p < end; p++) h = kco_rotl64(h ^ ((uint64_t)*p * KCO_P64_5), 11) * KCO_P64_1;
    h ^= h >> 33;
    h *= KCO_P64_2;
    h ^= h >> 29;
    h *= KCO_P64_3;
    h ^= h >> 32;
    return h;
}

typedef struct {
    uint64_t lines, count_sum, hash_sum, hash_xor;
} digest;

static inline void digest_line(digest *d, const unsigned char *line, size_t len, uint64_t t) {
    const uint64_t h = xxh64(line, len, 0);
    d->lines++;
    d->count_sum += t;
    d->hash_sum += h;
    d->hash_xor ^= h;
}
static void digest_add(digest *d, const digest *o) {
    d->lines += o->lines;
    d->count_sum += o->count_sum;
    d->hash_sum += o->hash_sum;
    d->hash_xor ^= o->hash_xor;
}
static void print_digest(const digest *d, const char *extra) {
    printf("{\"lines\": %llu, \"count_sum\": %llu, \"hash_sum\": \"%016llx\", \"hash_xor\": \"%016llx\"%s}\n",
           (unsigned long long)d->lines, (unsigned long long)d->count_sum, (unsigned long long)d->hash_sum,
           (unsigned long long)d->hash_xor, extra ? extra : "");
}

/* ---- lines: digest of an output file ---------------------------------------------------- */
static int cmd_lines(int argc, char **argv) {
    FILE *f = stdin;
    if (argc >= 3 && strcmp(argv[2], "-")) {
        f = fopen(argv[2], "rb");
        if (!f) { fprintf(stderr, "cannot open %s: %s\n", argv[2], strerror(errno)); return 1; }
    }
    const size_t cap = 64u << 20;
    unsigned char *buf = (unsigned char *)malloc(cap);
    size_t have = 0, n;
    digest d = {0, 0, 0, 0};
    for (;;) {
        n = fread(buf + have, 1, cap - have, f);
        have += n;
        size_t pos = 0;
        for (;;) {
            unsigned char *nl = (unsigned char *)memchr(buf + pos, '\n', have - pos);
            if (!nl) break;
            const size_t len = (size_t)(nl - (buf + pos)) + 1;
            uint64_t t = 0, mul = 1;
            for (const unsigned char *q = nl - 1; q >= buf + pos && *q != ' '; q--) {
                t += (uint64_t)(*q - '0') * mul;
                mul *= 10;
            }
            digest_line(&d, buf + pos, len, t);
            pos += len;
        }
        memmove(buf, buf + pos, have - pos);
        have -= pos;
        if (n == 0) {
            if (have) { fprintf(stderr, "unterminated last line\n"); return 1; }
            break;
        }
    }
    if (f != stdin) fclose(f);
    free(buf);
    print_digest(&d, NULL);
    return 0;
}

/* ---- count: partitioned restatement count ----------------------------------------------- */
typedef struct {
    uint64_t *slot; /* cap slots of nw key words + 1 count word (0 = empty): one cache line per probe */
    uint64_t cap, n;
    int nw;
} ptable;

static void pt_init(ptable *t, int nw, uint64_t cap) {
    t->nw = nw;
    t->cap = cap;
    t->n = 0;
    t->slot = (uint64_t *)calloc(cap * (nw + 1), sizeof(uint64_t));
    if (!t->slot) { fprintf(stderr, "out of memory (%llu slots)\n", (unsigned long long)cap); exit(1); }
}
static void pt_free(ptable *t) { free(t->slot); }
static void pt_add(ptable *t, const uint64_t *key, uint64_t h, uint64_t inc);
static void pt_grow(ptable *t) {
    ptable o = *t;
    pt_init(t, o.nw, o.cap * 2);
    for (uint64_t i = 0; i < o.cap; i++) {
        const uint64_t *s = o.slot + i * (o.nw + 1);
        if (s[o.nw]) pt_add(t, s, kco_key_hash((const kco_key *)s, o.nw), s[o.nw]);
    }
    pt_free(&o);
}
/* (kco_key_hash reads only the first nw words of its argument) */
static void pt_add(ptable *t, const uint64_t *key, uint64_t h, uint64_t inc) {
    if (4 * (t->n + 1) > 3 * t->cap) pt_grow(t);
    const int nw = t->nw;
    uint64_t i = h & (t->cap - 1);
    for (;;) {
        uint64_t *s = t->slot + i * (nw + 1);
        if (!s[nw]) {
            memcpy(s, key, nw * sizeof(uint64_t));
            s[nw] = inc;
            t->n++;
            return;
        }
        if (!memcmp(s, key, nw * sizeof(uint64_t))) {
            s[nw] += inc;
            return;
        }
        i = (i + 1) & (t->cap - 1);
    }
}

typedef struct {
    const unsigned char *file;
    const kco_chunk_list *chunks;
    int k, fmt, mode, parts, threads;
    uint64_t a;
    /* per thread */
    int tid;
    ptable tab;
    int part;
    /* keys of the partition waiting for their slot's cache line (prefetched when queued) */
    uint64_t q_key[16][4], q_h[16];
    int q_n, q_head;
    uint64_t windows, distinct;
    digest d;
} job;

/* partition of a canonical key: a cheap multiply-fold of its words, taken before the table hash
 * (which only the keys of the current partition pay) */
static inline int part_of(const uint64_t *w, int nw, int parts) {
    uint64_t x = w[nw - 1];
    for (int i = 0; i + 1 < nw; i++) x ^= w[i] * (0x9E3779B97F4A7C15ULL + 2 * (uint64_t)i);
    x *= 0xD6E8FEB86659FD93ULL;
    x ^= x >> 29;
    return (int)(((x >> 32) * (uint64_t)parts) >> 32);
}

static void on_kmer(void *vctx, const kco_roller *r) {
    job *j = (job *)vctx;
    const kco_key *canon = kco_key_cmp(&r->fwd, &r->rc, r->nw) <= 0 ? &r->fwd : &r->rc;
    if (part_of(canon->w, r->nw, j->parts) != j->part) return;
    pt_add(&j->tab, canon->w, kco_key_hash(canon, r->nw), 1);
}

/* kco_scan_chunk (kc_oracle_core.h: hash_kmers, parallel_parser.hpp:1322-1465) with the roller of
 * kco_roller_push (kmer_factory.cpp:172-239) unrolled for a constant word count: the same windows
 * and canonical keys, ~4x faster at the sizes the whole-job digests need (tests/test_oracle.py
 * checks it against kc_oracle's output on every golden case). */
#define KD_INLINE static inline __attribute__((always_inline))
KD_INLINE uint64_t scan_nw(job *j, const unsigned char *buf, uint64_t n, int bh, const int nw) {
    const int k = j->k, fmt = j->fmt, topbits = 2 * k - 64 * (nw - 1);
    const uint64_t topmask = topbits == 64 ? ~0ULL : ((1ULL << topbits) - 1);
    uint64_t f[4] = {0, 0, 0, 0}, rc[4] = {0, 0, 0, 0}, windows = 0;
    int fill = 0, parsing_header = bh;
    uint64_t i = 0;
    while (i < n) {
        const unsigned char ch = buf[i];
        if (fmt == KCO_FASTA) {
            if (ch == '>') parsing_header = 1;
            if (parsing_header) {
                while (i < n && buf[i] != '\n') i++;
                i++;
                parsing_header = 0;
                fill = 0;
                continue;
            }
            if (ch == '\n') { i++; continue; }
        }
        const int c = kco_char2int(ch);
        i++;
        if (c > 3) { fill = 0; continue; }
        if (fill == 0) {
            for (int q = 0; q < nw; q++) f[q] = rc[q] = 0;
        }
        for (int q = 0; q < nw - 1; q++) f[q] = (f[q] << 2) | (f[q + 1] >> 62);
        f[nw - 1] = (f[nw - 1] << 2) | (uint64_t)c;
        f[0] &= topmask;
        for (int q = nw - 1; q >= 1; q--) rc[q] = (rc[q] >> 2) | (rc[q - 1] << 62);
        rc[0] = (rc[0] >> 2) | ((uint64_t)(3 - c) << (topbits - 2));
        if (fill < k) fill++;
        if (fill < k) continue;
        windows++;
        int fwd = 1;
        for (int q = 0; q < nw; q++)
            if (f[q] != rc[q]) { fwd = f[q] < rc[q]; break; }
        const uint64_t *canon = fwd ? f : rc;
        if (part_of(canon, nw, j->parts) != j->part) continue;
        const uint64_t h = kco_key_hash((const kco_key *)canon, nw);
        __builtin_prefetch(j->tab.slot + (h & (j->tab.cap - 1)) * (nw + 1), 1);
        if (j->q_n == 16) { /* the oldest queued key: its line has had 15 keys' time to arrive */
            pt_add(&j->tab, j->q_key[j->q_head], j->q_h[j->q_head], 1);
            j->q_head = (j->q_head + 1) & 15;
            j->q_n--;
        }
        const int tail = (j->q_head + j->q_n) & 15;
        for (int q = 0; q < nw; q++) j->q_key[tail][q] = canon[q];
        j->q_h[tail] = h;
        j->q_n++;
    }
    return windows;
}
static uint64_t scan_chunk(job *j, kco_roller *r, const unsigned char *buf, uint64_t n, int bh) {
    switch (r->nw) {
    case 1: return scan_nw(j, buf, n, bh, 1);
    case 2: return scan_nw(j, buf, n, bh, 2);
    case 3: return scan_nw(j, buf, n, bh, 3);
    case 4: return scan_nw(j, buf, n, bh, 4);
    default: return kco_scan_chunk(buf, n, bh, j->fmt, r, on_kmer, j);
    }
}

static void *worker(void *arg) {
    job *j = (job *)arg;
    kco_roller r;
    kco_roller_init(&r, j->k);
    pt_init(&j->tab, r.nw, 1u << 20);
    char *line = (char *)malloc((size_t)j->k + 32);
    kco_key key;
    memset(&key, 0, sizeof(key));
    for (j->part = j->tid; j->part < j->parts; j->part += j->threads) {
        uint64_t w = 0;
        for (size_t c = 0; c < j->chunks->n; c++)
            w += scan_chunk(j, &r, j->file + j->chunks->v[c].off, j->chunks->v[c].len, j->chunks->v[c].bh);
        for (; j->q_n; j->q_n--, j->q_head = (j->q_head + 1) & 15)
            pt_add(&j->tab, j->q_key[j->q_head], j->q_h[j->q_head], 1);
        j->windows = w; /* every partition's scan sees every window */
        for (uint64_t i = 0; i < j->tab.cap; i++) {
            const uint64_t *s = j->tab.slot + i * (r.nw + 1);
            if (!s[r.nw]) continue;
            j->distinct++;
            const uint64_t t = kco_transform(s[r.nw], j->mode);
            if (j->a == 0 || t < j->a) continue;
            memcpy(key.w, s, r.nw * sizeof(uint64_t));
            for (int p = 0; p < j->k; p++) line[p] = kco_int2char[kco_key_char(&key, j->k, r.nw, p)];
            const int len = j->k + sprintf(line + j->k, " %llu\n", (unsigned long long)t);
            digest_line(&j->d, (const unsigned char *)line, (size_t)len, t);
        }
        memset(j->tab.slot, 0, j->tab.cap * (r.nw + 1) * sizeof(uint64_t));
        j->tab.n = 0;
        fprintf(stderr, "kc_digest: partition %d of %d done (thread %d)\n", j->part + 1, j->parts, j->tid);
    }
    free(line);
    pt_free(&j->tab);
    return NULL;
}

static int detect_format(const char *path, const unsigned char *buf, uint64_t size) {
    /* file_format (main.cpp:27-68), as kc_oracle.c */
    const char *dot = strrchr(path, '.');
    const char *slash = strrchr(path, '/');
    if (dot && slash && dot < slash) dot = NULL;
    unsigned char first = size ? buf[0] : 0;
    if (dot && (!strcmp(dot, ".fasta") || !strcmp(dot, ".fa"))) return first == '>' ? '>' : -1;
    if (dot && (!strcmp(dot, ".fastq") || !strcmp(dot, ".fq"))) return first == '@' ? '@' : -1;
    return strchr("actgACGT", first) && first ? 0 : -1;
}

static int cmd_count(int argc, char **argv) {
    if (argc < 4) { fprintf(stderr, "usage: count INPUT K ...\n"); return 2; }
    const char *in = argv[2];
    int k = atoi(argv[3]), mode = 2, parts = 16, threads = 8;
    uint64_t a = 2, chunk = 10ull << 20;
    for (int i = 4; i < argc; i++) {
        if (!strcmp(argv[i], "-m")) mode = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-a")) a = strtoull(argv[++i], 0, 10);
        else if (!strcmp(argv[i], "-c")) chunk = strtoull(argv[++i], 0, 10);
        else if (!strcmp(argv[i], "-p")) parts = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-j")) threads = atoi(argv[++i]);
        else { fprintf(stderr, "unknown option %s\n", argv[i]); return 2; }
    }
    if (k < 1 || k > 32 * KCO_MAXW - 1 || parts < 1 || threads < 1) { fprintf(stderr, "bad arguments\n"); return 2; }
    if (threads > parts) threads = parts;
    int fd = open(in, O_RDONLY);
    if (fd < 0) { fprintf(stderr, "cannot open %s: %s\n", in, strerror(errno)); return 1; }
    struct stat st;
    fstat(fd, &st);
    const uint64_t size = (uint64_t)st.st_size;
    const unsigned char *file =
        size ? (const unsigned char *)mmap(NULL, size, PROT_READ, MAP_PRIVATE, fd, 0) : (const unsigned char *)"";
    if (file == MAP_FAILED) { fprintf(stderr, "mmap failed\n"); return 1; }
    int sym = detect_format(in, file, size);
    if (sym < 0) { fprintf(stderr, "Input file %s is ill-formed\n", in); return 1; }
    if (sym == '@') { fprintf(stderr, "Input file format not supported.\n"); return 1; }
    kco_chunk_list chunks = kco_make_chunks(file, size, k, chunk, (unsigned char)sym);
    job *jobs = (job *)calloc((size_t)threads, sizeof(job));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        memset(&jobs[t], 0, sizeof(job));
        jobs[t].file = file;
        jobs[t].chunks = &chunks;
        jobs[t].k = k;
        jobs[t].fmt = sym == '>' ? KCO_FASTA : KCO_PLAIN;
        jobs[t].mode = mode;
        jobs[t].parts = parts;
        jobs[t].threads = threads;
        jobs[t].a = a;
        jobs[t].tid = t;
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    digest d = {0, 0, 0, 0};
    uint64_t distinct = 0, windows = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        digest_add(&d, &jobs[t].d);
        distinct += jobs[t].distinct;
        windows = jobs[t].windows;
    }
    char extra[160];
    snprintf(extra, sizeof(extra), ", \"windows\": %llu, \"distinct\": %llu, \"parts\": %d",
             (unsigned long long)windows, (unsigned long long)distinct, parts);
    print_digest(&d, extra);
    free(chunks.v);
    free(jobs);
    free(th);
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 2 && !strcmp(argv[1], "lines")) return cmd_lines(argc, argv);
    if (argc >= 2 && !strcmp(argv[1], "count")) return cmd_count(argc, argv);
    fprintf(stderr, "usage: kc_digest lines [FILE|-] | count INPUT K [-m M] [-a A] [-c CHUNK] [-p PARTS] [-j THREADS]\n");
    return 2;
}
