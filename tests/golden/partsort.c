/*
 * partsort -- fixture-generation helper for tests/golden/make_fullsize.py (test
 * infrastructure, never part of the product path).
 *
 *   partsort IN DIR
 *
 * Streams the reference's output text (IN may be a FIFO the reference writes into) and
 * appends every line to DIR/<first three characters> (64 buckets over A < C < G < T), so
 * that sorting each bucket and concatenating the buckets in byte order gives the byte-sorted
 * file without holding it whole (the C5 share's output is ~78 GB).  Prints
 * "<lines> <sum of counts>" (the count is the token after the last space of each line).
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int code(int c) {
    switch (c) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    default: return -1;
    }
}

int main(int argc, char **argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: partsort IN DIR\n");
        return 2;
    }
    FILE *in = fopen(argv[1], "rb");
    if (!in) { perror(argv[1]); return 1; }
    FILE *out[65];
    static char names[65][4] = {{0}};
    for (int b = 0; b < 65; b++) {
        char path[4096];
        if (b < 64) {
            names[b][0] = "ACGT"[b >> 4];
            names[b][1] = "ACGT"[(b >> 2) & 3];
            names[b][2] = "ACGT"[b & 3];
        } else {
            strcpy(names[b], "zzz"); /* lines shorter than three characters (k < 3) */
        }
        snprintf(path, sizeof path, "%s/%s", argv[2], names[b]);
        out[b] = fopen(path, "wb");
        if (!out[b]) { perror(path); return 1; }
        setvbuf(out[b], NULL, _IOFBF, 1 << 20);
    }
    char *line = NULL;
    size_t cap = 0;
    ssize_t n;
    unsigned long long lines = 0, total = 0;
    while ((n = getline(&line, &cap, in)) > 0) {
        if (line[n - 1] != '\n') { fprintf(stderr, "unterminated last line\n"); return 1; }
        int b = 64;
        if (n >= 4) {
            int c0 = code(line[0]), c1 = code(line[1]), c2 = code(line[2]);
            if (c0 >= 0 && c1 >= 0 && c2 >= 0) b = (c0 << 4) | (c1 << 2) | c2;
        }
        char *sp = memrchr(line, ' ', (size_t)n);
        if (!sp) { fprintf(stderr, "line without a count\n"); return 1; }
        total += strtoull(sp + 1, NULL, 10);
        lines++;
        if (fwrite(line, 1, (size_t)n, out[b]) != (size_t)n) { perror("write"); return 1; }
    }
    for (int b = 0; b < 65; b++)
        if (fclose(out[b])) { perror("close"); return 1; }
    printf("%llu %llu\n", lines, total);
    return 0;
}
