/*
 * kc_gen -- CPU synthetic read generator (bench/test input tool).
 *   kc_gen OUT N L G [-s SEED] [-e ERR] [-n NRATE] [-w WRAP] [--first R0 --count RC] [--plain]
 *          [--homo FRAC] [--dinuc FRAC] [--repeat LEN COPIES]   (skewed workloads, kc_synth.h)
 * Writes FASTA records ">r<i>\n<seq>\n" (or plain "<seq>\n" lines with --plain)
 * identical to the device generator kc_synth_device() for the same parameters.
 */
#include "../csrc/kc_synth.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: kc_gen OUT N L G [-s SEED] [-e ERR] [-n NRATE] [-w WRAP] [--first R0] [--count RC] [--plain]\n");
        return 2;
    }
    kc_synth_params p;
    memset(&p, 0, sizeof(p));
    p.n_reads = strtoull(argv[2], 0, 10);
    p.read_len = (uint32_t)atoi(argv[3]);
    p.genome_len = strtoull(argv[4], 0, 10);
    p.seed = 42;
    p.err_rate = 0.001;
    uint64_t first = 0, count = ~0ULL;
    int plain = 0;
    for (int i = 5; i < argc; i++) {
        if (!strcmp(argv[i], "-s")) p.seed = strtoull(argv[++i], 0, 10);
        else if (!strcmp(argv[i], "-e")) p.err_rate = atof(argv[++i]);
        else if (!strcmp(argv[i], "-n")) p.n_rate = atof(argv[++i]);
        else if (!strcmp(argv[i], "-w")) p.wrap = (uint32_t)atoi(argv[++i]);
        else if (!strcmp(argv[i], "--first")) first = strtoull(argv[++i], 0, 10);
        else if (!strcmp(argv[i], "--count")) count = strtoull(argv[++i], 0, 10);
        else if (!strcmp(argv[i], "--plain")) plain = 1;
        else if (!strcmp(argv[i], "--homo")) p.homo_frac = atof(argv[++i]);
        else if (!strcmp(argv[i], "--dinuc")) p.dinuc_frac = atof(argv[++i]);
        else if (!strcmp(argv[i], "--repeat")) {
            p.repeat_len = (uint32_t)atoi(argv[++i]);
            p.repeat_copies = (uint32_t)atoi(argv[++i]);
        }
        else { fprintf(stderr, "unknown option %s\n", argv[i]); return 2; }
    }
    if (p.genome_len < p.read_len) { fprintf(stderr, "G < L\n"); return 2; }
    FILE *f = fopen(argv[1], "wb");
    if (!f) { perror(argv[1]); return 1; }
    static char buf[1 << 20];
    setvbuf(f, buf, _IOFBF, sizeof(buf));
    uint64_t e_th = kcs_thresh(p.err_rate), n_th = kcs_thresh(p.n_rate);
    uint64_t last = count == ~0ULL ? p.n_reads : first + count;
    if (last > p.n_reads) last = p.n_reads;
    char *seq = (char *)malloc(p.read_len + 1);
    static const char sym[5] = {'A', 'C', 'G', 'T', 'N'};
    for (uint64_t i = first; i < last; i++) {
        uint64_t st = kcs_read_start(&p, i);
        int rc = kcs_read_rc(&p, i);
        for (uint32_t j = 0; j < p.read_len; j++) seq[j] = sym[kcs_read_base(&p, i, j, st, rc, e_th, n_th)];
        if (!plain) fprintf(f, ">r%llu\n", (unsigned long long)i);
        if (p.wrap && !plain) {
            for (uint32_t j = 0; j < p.read_len; j += p.wrap) {
                uint32_t n = p.read_len - j < p.wrap ? p.read_len - j : p.wrap;
                fwrite(seq + j, 1, n, f);
                fputc('\n', f);
            }
        } else {
            fwrite(seq, 1, p.read_len, f);
            fputc('\n', f);
        }
    }
    fclose(f);
    free(seq);
    return 0;
}
