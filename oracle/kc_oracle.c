/*
 * kc_oracle -- CLI around kc_oracle_core.h (the CPU parity checker).
 *
 * TEST INFRASTRUCTURE ONLY: executed by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg, never by the product.  See kc_oracle_core.h.
 *
 *   kc_oracle count  INPUT K [-m M] [-a A] [-s S] [-b -u U [-f F]] [-c CHUNK] -o OUT
 *       Sorted "<CANONICAL_KMER> <T(c)>" lines for T(c) >= A (A = 0: no file),
 *       the result contract of the reference.  Prints
 *       "windows=<W> distinct=<D> passed=<P> new_in_second=<N>" on stdout.
 *   kc_oracle chunks INPUT K [-c CHUNK]      reference chunk table: "off len bh"
 *   kc_oracle xxh64  SEED V...               XXH64(&v, 8, seed) per value
 *   kc_oracle root   K SEQ                   Rabin-Karp mod 2^54 root of a k-mer
 */
#include "kc_oracle_core.h"

#include <errno.h>
#include <sys/stat.h>
#include <time.h>

static unsigned char *read_file(const char *path, uint64_t *size) {
    FILE *f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "cannot open %s: %s\n", path, strerror(errno)); exit(1); }
    struct stat st;
    fstat(fileno(f), &st);
    *size = (uint64_t)st.st_size;
    unsigned char *b = (unsigned char *)malloc(*size + 1);
    if (*size && fread(b, 1, *size, f) != *size) { fprintf(stderr, "short read\n"); exit(1); }
    fclose(f);
    return b;
}

/* file_format (main.cpp:27-68): extension .fasta/.fa -> FASTA, .fastq/.fq -> FASTQ
 * (unsupported), else one-string-per-line.  Returns start symbol, -1 ill-formed. */
static int detect_format(const char *path, const unsigned char *buf, uint64_t size) {
    const char *dot = strrchr(path, '.');
    const char *slash = strrchr(path, '/');
    if (dot && slash && dot < slash) dot = NULL;
    unsigned char first = size ? buf[0] : 0;
    if (dot && (!strcmp(dot, ".fasta") || !strcmp(dot, ".fa"))) return first == '>' ? '>' : -1;
    if (dot && (!strcmp(dot, ".fastq") || !strcmp(dot, ".fq"))) return first == '@' ? '@' : -1;
    return strchr("actgACGT", first) && first ? 0 : -1;
}

typedef struct {
    kco_counter *cnt;
    kco_bloom *bf;
    int pass;            /* 0 = count, 1 = bloom pass 1, 2 = count behind bloom gate */
    uint64_t passed;
} scan_ctx;

static void on_kmer(void *vctx, const kco_roller *r) {
    scan_ctx *s = (scan_ctx *)vctx;
    const kco_key *canon = kco_key_cmp(&r->fwd, &r->rc, r->nw) <= 0 ? &r->fwd : &r->rc;
    if (s->pass >= 1) {
        uint64_t f = kco_rk54(&r->fwd, r->k, r->nw), b = kco_rk54(&r->rc, r->k, r->nw);
        uint64_t root = f < b ? f : b;
        if (s->pass == 1) { kco_bloom_insert(s->bf, root); return; }
        if (!kco_bloom_gate(s->bf, root)) return;
    }
    s->passed++;
    kco_counter_add(s->cnt, canon, 1);
}

static int cmp_idx_nw;
static const kco_key *cmp_keys;
static int cmp_idx(const void *a, const void *b) {
    return kco_key_cmp(&cmp_keys[*(const uint64_t *)a], &cmp_keys[*(const uint64_t *)b], cmp_idx_nw);
}

static int cmd_count(int argc, char **argv) {
    if (argc < 4) { fprintf(stderr, "usage: count INPUT K ...\n"); return 2; }
    const char *in = argv[2];
    int k = atoi(argv[3]);
    int mode = 2, use_bf = 0;
    uint64_t a = 2, U = 0, chunk = 10ull << 20;
    double fpr = 0.01;
    const char *out = NULL;
    for (int i = 4; i < argc; i++) {
        if (!strcmp(argv[i], "-m")) mode = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-a")) a = strtoull(argv[++i], 0, 10);
        else if (!strcmp(argv[i], "-s")) ++i; /* table size: irrelevant to the result */
        else if (!strcmp(argv[i], "-b")) use_bf = 1;
        else if (!strcmp(argv[i], "-u")) U = strtoull(argv[++i], 0, 10);
        else if (!strcmp(argv[i], "-f")) fpr = atof(argv[++i]);
        else if (!strcmp(argv[i], "-c")) chunk = strtoull(argv[++i], 0, 10);
        else if (!strcmp(argv[i], "-o")) out = argv[++i];
        else { fprintf(stderr, "unknown option %s\n", argv[i]); return 2; }
    }
    if (k < 1 || k > 32 * KCO_MAXW - 1) { fprintf(stderr, "k out of range\n"); return 2; }
    uint64_t size;
    unsigned char *buf = read_file(in, &size);
    int sym = detect_format(in, buf, size);
    if (sym < 0) { fprintf(stderr, "Input file %s is ill-formed\n", in); return 1; }
    if (sym == '@') { printf("Input file format not supported."); return 0; }
    int fmt = sym == '>' ? KCO_FASTA : KCO_PLAIN;
    kco_chunk_list chunks = kco_make_chunks(buf, size, k, chunk, (unsigned char)sym);
    kco_roller r;
    kco_roller_init(&r, k);
    kco_counter cnt;
    kco_counter_init(&cnt, r.nw, 1 << 16);
    kco_bloom bf;
    scan_ctx s = {&cnt, &bf, 0, 0};
    uint64_t windows = 0;
    if (use_bf) {
        kco_bloom_init(&bf, U, fpr);
        s.pass = 1;
        for (size_t c = 0; c < chunks.n; c++)
            kco_scan_chunk(buf + chunks.v[c].off, chunks.v[c].len, chunks.v[c].bh, fmt, &r, on_kmer, &s);
        /* -m 1 -b runs pass 1 and then ignores the filter (main.cpp:482-489) */
        s.pass = mode == 1 ? 0 : 2;
    }
    for (size_t c = 0; c < chunks.n; c++)
        windows += kco_scan_chunk(buf + chunks.v[c].off, chunks.v[c].len, chunks.v[c].bh, fmt, &r, on_kmer, &s);
    printf("windows=%llu distinct=%llu passed=%llu new_in_second=%llu chunks=%zu\n",
           (unsigned long long)windows, (unsigned long long)cnt.n, (unsigned long long)s.passed,
           (unsigned long long)(use_bf ? bf.new_in_second : 0), chunks.n);
    if (a > 0 && out) {
        uint64_t *idx = (uint64_t *)malloc((cnt.n + 1) * sizeof(uint64_t));
        uint64_t m = 0;
        for (uint64_t i = 0; i < cnt.cap; i++)
            if (cnt.used[i] && kco_transform(cnt.cnt[i], mode) >= a) idx[m++] = i;
        cmp_idx_nw = cnt.nw;
        cmp_keys = cnt.keys;
        qsort(idx, m, sizeof(uint64_t), cmp_idx);
        FILE *f = fopen(out, "wb");
        char *line = (char *)malloc((size_t)k + 32);
        for (uint64_t j = 0; j < m; j++) {
            const kco_key *key = &cnt.keys[idx[j]];
            for (int p = 0; p < k; p++) line[p] = kco_int2char[kco_key_char(key, k, cnt.nw, p)];
            int len = k + sprintf(line + k, " %llu\n", (unsigned long long)kco_transform(cnt.cnt[idx[j]], mode));
            fwrite(line, 1, (size_t)len, f);
        }
        fclose(f);
        free(line);
        free(idx);
    }
    if (use_bf) kco_bloom_free(&bf);
    kco_counter_free(&cnt);
    free(chunks.v);
    free(buf);
    return 0;
}

static int cmd_chunks(int argc, char **argv) {
    if (argc < 4) return 2;
    uint64_t chunk = 10ull << 20;
    for (int i = 4; i < argc; i++)
        if (!strcmp(argv[i], "-c")) chunk = strtoull(argv[++i], 0, 10);
    uint64_t size;
    unsigned char *buf = read_file(argv[2], &size);
    int sym = detect_format(argv[2], buf, size);
    if (sym < 0) return 1;
    kco_chunk_list l = kco_make_chunks(buf, size, atoi(argv[3]), chunk, (unsigned char)sym);
    for (size_t i = 0; i < l.n; i++)
        printf("%llu %llu %d\n", (unsigned long long)l.v[i].off, (unsigned long long)l.v[i].len, l.v[i].bh);
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: kc_oracle count|chunks|xxh64|root ...\n");
        return 2;
    }
    if (!strcmp(argv[1], "count")) return cmd_count(argc, argv);
    if (!strcmp(argv[1], "chunks")) return cmd_chunks(argc, argv);
    if (!strcmp(argv[1], "xxh64")) {
        uint64_t seed = strtoull(argv[2], 0, 0);
        for (int i = 3; i < argc; i++)
            printf("%llu\n", (unsigned long long)kco_xxh64_u64(strtoull(argv[i], 0, 0), seed));
        return 0;
    }
    if (!strcmp(argv[1], "root")) {
        int k = atoi(argv[2]);
        kco_roller r;
        kco_roller_init(&r, k);
        for (const char *p = argv[3]; *p; p++) kco_roller_push(&r, kco_char2int((unsigned char)*p));
        uint64_t f = kco_rk54(&r.fwd, k, r.nw), b = kco_rk54(&r.rc, k, r.nw);
        printf("%llu %llu %llu\n", (unsigned long long)f, (unsigned long long)b,
               (unsigned long long)(f < b ? f : b));
        return 0;
    }
    fprintf(stderr, "unknown command %s\n", argv[1]);
    return 2;
}
