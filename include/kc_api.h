/*
 * kc_api.h -- C ABI of the MI355X canonical k-mer counting engine
 * (canonical-k-mer-hash-table_amd/lib/libkc.so).
 *
 * This is the drop-in boundary for the hot path of Kaarme
 * (Denopia/canonical-k-mer-hash-table): parallel_parser -> kmer_factory ->
 * kmer_hash_table (+ double_bloomfilter).  The reference has no FFI; its internal
 * seams are the per-chunk worker call hash_kmers(chunk, format)
 * (include/parallel_parser.hpp:1302-1479), the per-k-mer table call
 * process_kmer_MT (include/kmer_hash_table.hpp:308, source/kmer_hash_table.cpp:2207)
 * and the writers (source/kmer_hash_table.cpp:2013-2050, 4318-4524).  Each entry
 * point below names the reference interface it replaces.
 *
 * Conventions: plain pointers and sizes, no C++ or torch types.  Every call
 * returns 0 (KC_OK) or a negative KC_ERR_*; the library never exit()s (the
 * reference does, e.g. kmer_hash_table.cpp:2552-2556) -- kc_last_error() gives
 * the message.  A context owns all device memory and is used by one host thread
 * at a time.  Host buffers passed to *_chunk calls are copied before return.
 */
#ifndef KC_API_H
#define KC_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Largest k-mer length: keys of up to fifteen 64-bit words, which with their count fill
   one 128-byte table bucket (the reference sizes its blocks dynamically,
   kmer_factory.cpp:33, and accepts any k > 0, main.cpp:135; INTEGRATION.md "Differences"
   states this bound). */
#define KC_MAX_K 479

#define KC_OK 0
#define KC_ERR_ARG (-1)         /* invalid argument */
#define KC_ERR_HIP (-2)         /* HIP runtime / device error */
#define KC_ERR_TABLE_FULL (-3)  /* "Hash table is full" (kmer_hash_table.cpp:2552-2556) */
#define KC_ERR_STATE (-4)       /* call out of order (e.g. count before bloom finalize) */
#define KC_ERR_IO (-5)          /* file error */
#define KC_ERR_NOMEM (-6)       /* host or device allocation failed */
#define KC_ERR_UNSUPPORTED (-7) /* the Bloom filter on the per-window routing entry point kc_route_device (a sharded
                                   Bloom job routes {key, count} records to the filter's owner instead:
                                   kc_bloom_records_device); the compact representation of a -m 0 table */

/* input_mode of main.cpp:178-189 */
#define KC_FMT_FASTA 0
#define KC_FMT_FASTQ 1
#define KC_FMT_PLAIN 2

typedef struct kc_ctx kc_ctx;

/* Replaces the CLI-derived arguments struct (main.cpp:70-99) that main() hands to
 * the parse_input_* functors (main.cpp:468-543). */
typedef struct {
    int32_t k;              /* KLEN, 1..KC_MAX_K (the reference is wrong for k % 32 == 0) */
    int32_t mode;           /* -m: 0 plain table (uint16 counts wrap), 1/2 kaarme (saturate at 16383) */
    int32_t bf_enable;      /* -b: two-pass double Bloom filter prefilter */
    int32_t device;         /* HIP device ordinal */
    uint64_t table_slots;   /* -s: minimum hash table slots (ignored with bf_enable: 2 * new_in_second) */
    uint64_t est_unique;    /* -u: estimated unique k-mers, sizes the Bloom filter */
    double fpr;             /* -f: Bloom filter false positive rate (0.001..0.999) */
    uint64_t min_abundance; /* -a: output threshold on T(c) */
    uint64_t batch_bytes;   /* staging batch size in bytes (0 = 256 MiB) */
} kc_config;

/* One reference chunk (text_chunk, include/text_reader.h:17-36): `len` bytes at
 * `off` of a file image, processed with `broken_header`. */
typedef struct {
    uint64_t off;
    uint64_t len;
    int32_t broken_header;
    int32_t pad;
} kc_chunk;

typedef struct {
    uint64_t windows;         /* k-mer windows of the counting pass */
    uint64_t inserted;        /* windows inserted (all windows without BF; gate-passing with BF) */
    uint64_t distinct;        /* occupied table slots ("Main array slots used", parallel_parser.hpp:1551-1562) */
    uint64_t table_slots;     /* slot capacity of the device table */
    uint64_t bf_windows;      /* k-mer windows of Bloom pass 1 */
    uint64_t bf_bits;         /* bits per Bloom filter (main.cpp:402-418) */
    uint64_t new_in_first;    /* DoubleAtomicDoubleBloomFilter counters (double_bloomfilter.hpp:233-246) */
    uint64_t new_in_second;
    uint64_t failed_in_first;
    uint64_t chunks;          /* chunks processed by the counting pass */
    uint64_t bytes;           /* input bytes processed by the counting pass */
    uint64_t part_fallbacks;  /* partitioned batches redone on the exact layout (a full skew list) */
    uint64_t spilled;         /* keys past their segment's end, inserted through the exact levels */
    uint64_t heavy_records;   /* {k-mer, count} records of repeated windows (homopolymer runs) */
    uint64_t reused_passes;   /* counting passes that started from the Bloom pass's kept partitions */
    uint64_t reuse_level;     /* the partition level the last reused pass started from: 2 (level 3 only),
                                 1 (levels 2-3), 0 = no reuse */
    uint64_t route_counts_kept; /* kc_route_table_device calls that took the per-block owner counts the
                                   counting passes kept (kc_route_hint) instead of running a count pass */
    uint64_t deferred_level3;   /* level-3 passes of counting passes over several staging batches that
                                   inserted a group of batches' level-2 partitions at once (one table
                                   sweep per group, not per batch; KC_DEFER=0 disables it) */
} kc_stats;

/* Creates the device table (PointerHashTableCanonicalAV ctor,
 * kmer_hash_table.cpp:2128-2150 / BasicAtomicFlagHashTableLong, 1992-2003) and,
 * with bf_enable, the Bloom filter (DoubleAtomicDoubleBloomFilter ctor,
 * double_bloomfilter.hpp:255-260 sized as main.cpp:402-431). */
int kc_create(const kc_config* cfg, kc_ctx** out);
void kc_destroy(kc_ctx* ctx);
/* Message of the last failed call on ctx (or of kc_create when ctx == NULL). */
const char* kc_last_error(const kc_ctx* ctx);

/* Bloom pass 1 over one chunk: bloom_filter_kmers(chunk, format)
 * (parallel_parser.hpp:2788-2940) -> insertion_process per k-mer. */
int kc_bloom_chunk(kc_ctx* ctx, const uint8_t* buf, size_t len, int fmt, int broken_header);
/* End of pass 1: main.cpp:454-461 (min_slots = 2 * new_in_second; resize()).
 * Sizes and allocates the table. */
int kc_bloom_finalize(kc_ctx* ctx, uint64_t* new_in_second);
/* Counting pass over one chunk: hash_kmers(chunk, format) (parallel_parser.hpp:1302-1479)
 * calling process_kmer_MT per window (kmer_hash_table.cpp:2207) -- behind the Bloom
 * gate (parallel_parser.hpp:2436-2453) when bf_enable and mode != 1. */
int kc_count_chunk(kc_ctx* ctx, const uint8_t* buf, size_t len, int fmt, int broken_header);

/* The same two passes over a DEVICE-resident file image and a chunk table
 * (kc_plan_chunks), enqueued on hip_stream (a hipStream_t; NULL = the HIP null
 * stream) after the work already queued there, so a buffer produced on that stream
 * (e.g. by PyTorch on its current stream) is safe to pass.  The image must stay valid
 * until the work completes (kc_sync).  Every *_device entry point follows this rule.
 * Host waits inside these two calls (the work is still ordered on hip_stream):
 *   - an image that fits one staging batch (kc_config.batch_bytes): the call returns once
 *     the batch's single-pass levels have run -- it reads two device counters (skew list,
 *     segment overflow) to launch the batch's fallback work only when it is needed;
 *   - an image of several batches: before batch i+1 is queued, the call waits until batch i's
 *     chunk descriptors have reached the device (queued after the work before it), so at most
 *     one batch is queued ahead; the fallback work stays behind a device-side gate.  A counting
 *     pass of several batches defers level 3 (kc_stats.deferred_level3): the level-2 partitions
 *     of a group of batches wait in HBM and one level-3 pass inserts them (one sweep of the
 *     table per group, not per batch; KC_DEFER=0 disables it); the call then waits for each
 *     batch's partition levels (it reads the batch's skew-list and overflow counters);
 *   - the counting pass that reuses the Bloom pass's partitions waits for its work (below).
 * Level-1 reuse: when the Bloom pass is one staging batch, it keeps its window
 * partition, and a counting pass given the same image pointer, chunk table and format
 * -- and the same bytes, checked by a checksum of the chunks -- starts from that
 * partition instead of tokenizing and canonicalising every window again (that counting
 * call then waits for its work; kc_stats.reused_passes counts such passes).  Any
 * difference runs the ordinary counting pass.  KC_REUSE=0 disables it. */
int kc_bloom_device(kc_ctx* ctx, const uint8_t* dev_image, const kc_chunk* chunks, size_t n_chunks, int fmt,
                    void* hip_stream);
int kc_count_device(kc_ctx* ctx, const uint8_t* dev_image, const kc_chunk* chunks, size_t n_chunks, int fmt,
                    void* hip_stream);
/* Distinct-count estimate of a device image (no reference counterpart: Kaarme takes the
 * table size from its user, -s, main.cpp:134-154, or from the Bloom pass, main.cpp:454): the
 * canonical k-mers of the image's windows into a HyperLogLog sketch of 2^14 registers
 * (~0.8 % standard error; for k <= 128 over a 1/8 sample of the distinct k-mers picked by a
 * strand-symmetric hash, the estimate scaled by 8, whose sampling error is far smaller for
 * the millions of k-mers it is meant for and ~9 % at a thousand), so a caller can size a
 * table (kc_config.table_slots) before
 * counting, e.g. a rank's local table in a sharded job.  Counts nothing and leaves the
 * table alone; the call waits for its work (the estimate is a host value).  Any context of
 * the same k can run it (its table size does not matter).  When HBM allows, the context keeps
 * the tokenized batches (3/8 byte per input byte) for its next kc_count_device over the same
 * image pointer, chunk table and format, which then skips its tokenizer: the caller must not
 * change the image's bytes in between (kc_reset or any other pass drops them). */
int kc_estimate_distinct_device(kc_ctx* ctx, const uint8_t* dev_image, const kc_chunk* chunks, size_t n_chunks,
                                int fmt, void* hip_stream, double* estimate);
/* Size the device table of the job about to be counted (after kc_create or kc_reset, before
 * its first counting pass; no Bloom filter): `slots` k-mers with the usual 25 % headroom,
 * e.g. 1.1 x kc_estimate_distinct_device, instead of -s (kc_config.table_slots), which stays
 * the job's reference capacity (KC_STRICT_CAPACITY: kc_finish fails past next_prime3mod4(-s)).
 * 0 = back to -s.
 * A table much smaller than its allocation gets a new one (the memory goes back to the
 * deferred level 3).  Replaces nothing in the reference, whose table is -s slots
 * (parallel_parser.hpp:1192-1196): -s 2.6e9 for C4's 1.0 G distinct k-mers takes 83 GB of
 * HBM at 25 % headroom, the estimate 35 GB. */
int kc_size_table(kc_ctx* ctx, uint64_t slots);
/* Wait for all work enqueued on the context. */
int kc_sync(kc_ctx* ctx);

/* Multi-GPU hash-prefix sharding (the reference is single-process):
 * kc_route_device tokenizes a device image (its chunks must fit one staging batch) and
 * writes the table keys of its windows to dev_out grouped by owner shard (kc_key_words()
 * u64 per key, the engine's internal bijective key encoding); counts[d] = keys for
 * shard d.  out_capacity (keys) must be >= the image bytes + chunks.  The caller
 * exchanges the groups (all-to-all) and every owner inserts what it received with
 * kc_insert_keys_device.  Not available with the Bloom filter. */
int kc_route_device(kc_ctx* ctx, const uint8_t* dev_image, const kc_chunk* chunks, size_t n_chunks, int fmt,
                    uint32_t nshards, uint64_t* dev_out, uint64_t out_capacity, uint64_t* counts, void* hip_stream);
int kc_insert_keys_device(kc_ctx* ctx, const uint64_t* dev_keys, uint64_t n_keys, void* hip_stream);

/* Super-k-mer sharding (the multi-GPU exchange of kaarme_amd.sharded): the owner of
 * a canonical k-mer is a hash of its canonical minimizer (the least h(canonical m-mer) over its
 * k - m + 1 m-mers; m = 0: min(15, k)), the same for both strands, so every occurrence of a k-mer
 * has one owner and the owners' counts are exact.  kc_route_superkmers_device tokenizes a device
 * image (any number of staging batches) and writes, per owner o < nshards (<= 64), the maximal runs
 * of consecutive windows with owner o ("super-k-mers": a break symbol + the run's k - 1 + r symbols)
 * as a packed symbol stream -- pk words of 32 2-bit symbols, bk words of their break flags (bit 31 =
 * the word's first symbol), the tokenizer's layout -- into region o of dev_pk / dev_bk (cap_words
 * words per region, region o at o * cap_words); words[o] = words written (or needed), windows[o] =
 * windows routed.  cap_words = 0: a dry run that only sizes the regions; a region too small fails
 * with KC_ERR_NOMEM and words[] holding the sizes needed.  The caller exchanges region o with
 * rank o (all-to-all), and each owner counts what it received with kc_count_packed_device (or runs
 * its Bloom pass 1 over it with kc_bloom_packed_device, then kc_bloom_finalize and the counting
 * pass): the concatenated streams of every sender, n_words words, readable for n_words + 2 words;
 * `windows` = the windows they hold (sizes the partition levels; 0 = unknown).  Replaces the
 * reference's one shared table (kmer_hash_table.cpp:2207-2567) with one table per owner. */
int kc_route_superkmers_device(kc_ctx* ctx, const uint8_t* dev_image, const kc_chunk* chunks, size_t n_chunks,
                               int fmt, uint32_t nshards, int m, uint64_t* dev_pk, uint32_t* dev_bk,
                               uint64_t cap_words, uint64_t* words, uint64_t* windows, void* hip_stream);
int kc_count_packed_device(kc_ctx* ctx, const uint64_t* dev_pk, const uint32_t* dev_bk, uint64_t n_words,
                           uint64_t windows, void* hip_stream);
int kc_bloom_packed_device(kc_ctx* ctx, const uint64_t* dev_pk, const uint32_t* dev_bk, uint64_t n_words,
                           uint64_t windows, void* hip_stream);

/* Pre-aggregated sharding (the multi-GPU path of kaarme_amd.sharded): every rank counts
 * its own input into its own table, then kc_route_table_device writes the table's
 * occupied slots as records {W table-key words, raw count} grouped by owner shard
 * (the owner_of bit field of word 0) into dev_out (capacity in records; NULL = counts
 * only) and the per-owner record counts into counts[nshards] (nshards <= 64); after
 * the exchange kc_insert_counts_device adds received records into the owner's table.
 * Replaces the reference's single shared table (kmer_hash_table.cpp:2207-2567): the union
 * of the owners' tables is the count of the whole input. */
int kc_route_table_device(kc_ctx* ctx, uint32_t nshards, uint64_t* dev_out, uint64_t out_capacity,
                          uint64_t* counts, void* hip_stream);
/* Tells the context that its table will be routed to nshards (1..64) owners (0 = off): every
 * level-3 pass of the counting pipeline then also writes its region's record counts per owner
 * (the two 256-bucket blocks the route reads), so a kc_route_table_device(nshards) after
 * counting passes that all went through level 3 (the partitioned path; not the direct
 * small-batch path or the merge inserts) runs no count pass over the table -- one streaming
 * read of the table fewer per merge.  kc_stats.route_counts_kept counts
 * such routes.  The records and counts are the same either way. */
int kc_route_hint(kc_ctx* ctx, uint32_t nshards);
int kc_insert_counts_device(kc_ctx* ctx, const uint64_t* dev_records, uint64_t n_records, void* hip_stream);
/* The same for records that arrive as ngroups (<= 64) consecutive groups of
 * group_counts[g] records (host array), one per sending rank, each in the order
 * kc_route_table_device wrote it: sorted by region when the sender's table has this
 * table's size.  The table is then updated in one LDS pass per region over the groups'
 * region runs (no partition levels); groups that are not sorted take
 * kc_insert_counts_device. */
int kc_insert_counts_runs_device(kc_ctx* ctx, const uint64_t* dev_records, const uint64_t* group_counts,
                                 uint32_t ngroups, void* hip_stream);

/* Whole-filter primitives (the reference has one filter,
 * DoubleAtomicDoubleBloomFilter, double_bloomfilter.hpp:233-260, filled by every worker of
 * the Bloom pass, parallel_parser.hpp:2788-2940), for a caller that runs kc_bloom_device on
 * every rank and combines the ranks' whole filters itself.  (kaarme_amd.sharded does not: it
 * shards the filter by the k-mers' owner, kc_bloom_records_device / kc_count_records_device
 * below, so no filter crosses xGMI.)  The primitives:
 *   kc_bloom_get_device   copies words [first_word, first_word + n_words) of the filter to
 *                         dev_dst (after the work queued on hip_stream and the context);
 *   kc_bloom_merge_device combines nparts copies of one word range (consecutive in
 *                         dev_parts, n_words each; whole 16-word blocks in the blocked
 *                         layout) into dev_out: filter 1 = OR, filter 2 = OR | (filter-1
 *                         bits set in >= 2 copies), so every k-mer seen twice in the whole
 *                         input passes the gate (seen twice on one rank, or on two ranks);
 *   kc_bloom_set_device   replaces the whole filter (n_words = kc_bloom_info's count) and
 *                         sets the pass-1 counter new_in_second, which kc_bloom_finalize
 *                         sizes the table from (main.cpp:454), to kc_bloom_estimate of the
 *                         new filter (also returned in *new_in_second; the same on every rank
 *                         for the combined filter); new_in_first / failed_in_first stay the
 *                         rank's own;
 *   kc_bloom_estimate     the number of distinct k-mers in filter 2 estimated from its set
 *                         bits (X of m bits, h pass-1 positions: -(m/h) ln(1 - X/m)). */
int kc_bloom_get_device(kc_ctx* ctx, uint32_t* dev_dst, uint64_t first_word, uint64_t n_words, void* hip_stream);
int kc_bloom_merge_device(kc_ctx* ctx, const uint32_t* dev_parts, uint32_t nparts, uint64_t n_words,
                          uint32_t* dev_out, void* hip_stream);
int kc_bloom_set_device(kc_ctx* ctx, const uint32_t* dev_src, uint64_t n_words, uint64_t* new_in_second,
                        void* hip_stream);
int kc_bloom_estimate(kc_ctx* ctx, uint64_t* distinct_in_second, void* hip_stream);

/* Owner-sharded Bloom filter ("the BF is sharded by the same owner"): the two
 * passes of a Bloom job over pre-aggregated records {W table-key words, raw count} -- what
 * kc_route_table_device writes from an ungated local count and the exchange delivers to the
 * k-mers' owner -- on the owner's context (its filter sized for its 1/G share of -u):
 *   kc_bloom_records_device   Bloom pass 1 (before kc_bloom_finalize) over records of
 *                             DISTINCT keys (the senders' records of one k-mer summed first:
 *                             kaarme_amd.sharded aggregates them in a table): insertion_process
 *                             (double_bloomfilter.hpp:371-413) twice for a record of count >= 2
 *                             -- a k-mer seen at least twice sets its filter-2 bits -- then once
 *                             for every record of count 1, as in one sequential order of the
 *                             reference's pass (parallel_parser.hpp:2788-2940), so a singleton
 *                             meets one filter;
 *   kc_count_records_device   the counting pass (after kc_bloom_finalize, which sizes the table
 *                             2 * new_in_second, main.cpp:454): adds each record's count when
 *                             its filter-2 bits pass the gate (parallel_parser.hpp:2436-2453);
 *                             -m 1 -b and contexts without the filter add every record.
 * Blocked filter layout only (the reference layout hashes the Rabin-Karp root, which a table
 * key does not carry): KC_ERR_ARG otherwise. */
int kc_bloom_records_device(kc_ctx* ctx, const uint64_t* dev_records, uint64_t n_records, void* hip_stream);
int kc_count_records_device(kc_ctx* ctx, const uint64_t* dev_records, uint64_t n_records, void* hip_stream);

/* Kaarme's compact representation: PointerHashTableCanonicalAV's 8-byte
 * slot words (OneCharacterAndPointerKMerAtomicVariable, kmer.hpp:103-149: occupied, predecessor
 * exists, self / predecessor canonical during insertion, left and right character, 14-bit count,
 * 38-bit predecessor slot) plus a secondary array of the chain starts' full keys, built from the
 * counted table after the counting pass (the reference builds it while inserting,
 * kmer_hash_table.cpp:2207-2567).  Every k-mer links to a k-mer of the table that precedes it on
 * the strand its minimizer reads forward, so the reference's walk (reconstruct_kmer_in_slot,
 * kmer_hash_table.cpp:3848-4058) rebuilds it in at most k - 2 hops.  -m 1 / -m 2 only (14-bit
 * counts); a snapshot: later counting does not update it, kc_reset drops it.
 *   kc_compact        builds it at the given load (slots = k-mers / load; 0 = 0.8);
 *   kc_compact_dump   reconstructs every k-mer with T(c) >= a: records as kc_dump, plus the
 *                     longest and the mean walk (hops);
 *   kc_compact_lookup T(c) of canonical keys (host arrays, kc_key_words() words each, the
 *                     kc_dump key layout) from the compact words alone, 0 if absent;
 *   kc_compact_read   copies the slot words and the secondary array's words to the host. */
typedef struct {
    uint64_t slots;         /* slot words (8 bytes each) */
    uint64_t kmers;         /* k-mers held (the table's distinct k-mers) */
    uint64_t chain_starts;  /* k-mers without a predecessor: full keys in the secondary array */
    uint64_t bytes;         /* slot words + secondary array */
    uint64_t table_bytes;   /* the full-key table it was built from */
} kc_compact_info;
int kc_compact(kc_ctx* ctx, double load, kc_compact_info* info);
int kc_compact_dump(kc_ctx* ctx, uint64_t** records, uint64_t* n_records, uint64_t* max_hops, double* mean_hops);
int kc_compact_lookup(kc_ctx* ctx, const uint64_t* keys, uint64_t n, uint32_t* counts);
int kc_compact_read(kc_ctx* ctx, uint64_t* words, uint64_t n_words, uint64_t* second, uint64_t n_second_words);

/* Re-initialise the table, the Bloom filter and all counters (the table/filter
 * constructors again, without reallocating). */
int kc_reset(kc_ctx* ctx);

/* Empty the table only (the next pass that touches it zero-fills it first), keeping the
 * job's counters (windows, chunks, bytes, ...).  The sharded front end calls it on a
 * rank's local table once kc_route_table_device has copied the table out, so the next
 * merge routes only what was counted since (the reference has one shared table and no
 * such step: kmer_hash_table.cpp:2207-2567). */
int kc_clear_table(kc_ctx* ctx);

/* Per-kernel device time, accumulated while profiling is enabled (HIP events on
 * the stream each kernel runs on). */
typedef struct {
    double gather_ms;      /* k_gather (device-image path only) */
    double tokenize_ms;    /* k_tile_summary + k_tile_scan + k_emit */
    double count_ms;       /* k_count (table insert / Bloom pass / gated insert) */
    uint64_t launches;     /* batches timed */
    uint64_t symbols;      /* symbol-stream bytes produced by the timed batches */
} kc_timing;
int kc_profile(kc_ctx* ctx, int enable);
int kc_get_timing(kc_ctx* ctx, kc_timing* t);  /* waits for the timed work; resets the accumulators */

/* Flush staged chunks, wait, and report counters (the timers/counters the functors
 * print, parallel_parser.hpp:1544-1562). stats may be NULL. */
int kc_finish(kc_ctx* ctx, kc_stats* stats);

/* Records {key words[kc_key_words()], T(c)} for every k-mer with T(c) >= a, in
 * table order; key word 0 is most significant, character j of the k-mer is bits
 * 2(k-1-j)..2(k-1-j)+1 of the 64*W-bit integer.  T(c) = c mod 65536 for -m 0,
 * min(c, 16383) otherwise.  Free with kc_free. */
int kc_dump(kc_ctx* ctx, uint64_t** records, uint64_t* n_records);
/* Writes "<CANONICAL_KMER> <T(c)>\n" lines for T(c) >= a (a == 0: nothing written):
 * write_kmers_on_disk_separately_even_faster (kmer_hash_table.cpp:4318-4524) /
 * write_kmers (2013-2050).  Line order is unspecified, as in the reference. */
int kc_write(kc_ctx* ctx, const char* path);
/* Order-independent digest of the text kc_write would write (the reference has none; its
 * output order is unspecified): every line "<CANONICAL_KMER> <T(c)>\n" is
 * hashed with XXH64 (seed 0) over its bytes incl. the '\n'; hash_sum is the sum of those
 * hashes mod 2^64 and hash_xor their XOR.  Any line order gives the same digest, and the digests
 * of disjoint line sets add up (lines, count_sum, hash_sum by addition mod 2^64, hash_xor by XOR),
 * so the owners of a sharded job combine theirs into the whole job's, comparable with a digest of
 * the reference's output file (oracle/kc_digest.c lines).  a == 0: all zero (no output). */
typedef struct {
    uint64_t lines;      /* lines (k-mers with T(c) >= a) */
    uint64_t count_sum;  /* sum of T(c) over the lines */
    uint64_t hash_sum;   /* sum of XXH64(line) mod 2^64 */
    uint64_t hash_xor;   /* XOR of XXH64(line) */
} kc_digest;
int kc_output_digest(kc_ctx* ctx, kc_digest* out);
int kc_key_words(const kc_ctx* ctx);
void kc_free(void* p);

/* Reference chunking of a file image: io_worker (parallel_parser.hpp:1230-1299) +
 * read_chunk_from_file (text_reader.h:93-226) with chunk_size (0 = 10 MiB,
 * main.cpp:387).  *chunks is allocated by the library (kc_free). */
int kc_plan_chunks(const uint8_t* image, uint64_t size, int k, uint64_t chunk_size, int fmt, kc_chunk** chunks,
                   uint64_t* n_chunks);
/* The same chunk table for an image in device memory (after the device's queued work): the
 * planner reads only the bytes around chunk ends, copied to the host in 64 KiB pages on demand,
 * instead of the caller copying the whole image to the host first. */
int kc_plan_chunks_device(const uint8_t* dev_image, uint64_t size, int k, uint64_t chunk_size, int fmt,
                          kc_chunk** chunks, uint64_t* n_chunks);

/* The reference's table size for a minimum of `min_slots` slots: the next prime that is
 * 3 mod 4 (next_prime3mod4, functions_math.cpp:53-96; "Hash table size is:").  The device
 * table keeps 25 % headroom over it (open addressing inside LDS-sized regions), so a job
 * whose distinct k-mers fall between the two succeeds where the reference exits with
 * "Hash table is full"; with KC_STRICT_CAPACITY=1 in the environment (CLI:
 * --strict-capacity) kc_finish returns KC_ERR_TABLE_FULL there too. */
uint64_t kc_table_size_reference(uint64_t min_slots);

/* Test hooks for the Bloom filter (not on the reference's path).
 * kc_xxh64: XXH64(&values[i], 8, seeds[i]) computed by the device function the
 *   reference-layout Bloom passes use (calculate_hashes, double_bloomfilter.hpp:276-281;
 *   xxHash v0.8.2), host arrays in and out.
 * kc_bloom_info: the filter's geometry: words (u32) of its bit array, filter bits per
 *   filter (main.cpp:402-418), ceil(hf) pass-1 and trunc(hf) pass-2 positions
 *   (main.cpp:417, parallel_parser.hpp:2397), layout 1 = blocked (default), 0 = reference.
 * kc_bloom_read / kc_bloom_write: copy the filter's words to / from the host (a write
 *   makes the next pass read the given bits). */
int kc_xxh64(const uint64_t* values, const uint64_t* seeds, uint64_t n, uint64_t* out);
int kc_bloom_info(kc_ctx* ctx, uint64_t* n_words, uint64_t* bits, int* nh, int* nh_gate, int* layout);
int kc_bloom_read(kc_ctx* ctx, uint32_t* words, uint64_t n_words);
int kc_bloom_write(kc_ctx* ctx, const uint32_t* words, uint64_t n_words);

/* Synthetic reads (bench/test input): writes the FASTA records
 * [first_read, first_read + n_reads) of the seeded generator to device memory
 * dev_dst (which receives kc_synth_bytes(first_read, n_reads) bytes). */
uint64_t kc_synth_bytes(uint64_t first_read, uint64_t n_reads, uint32_t read_len, uint32_t wrap);
int kc_synth_device(uint8_t* dev_dst, uint64_t first_read, uint64_t n_reads, uint64_t seed, uint64_t genome_len,
                    uint32_t read_len, uint32_t wrap, double err_rate, double n_rate, void* hip_stream);
/* Skewed variant (bench workloads and skew tests; kc_gen --homo/--dinuc/--repeat):
 * fractions of homopolymer and (CA)n reads, and a repeat of repeat_len bases present
 * repeat_copies times in the genome. */
typedef struct {
    double homo_frac;
    double dinuc_frac;
    uint32_t repeat_len;
    uint32_t repeat_copies;
} kc_synth_skew;
int kc_synth_skew_device(uint8_t* dev_dst, uint64_t first_read, uint64_t n_reads, uint64_t seed, uint64_t genome_len,
                         uint32_t read_len, uint32_t wrap, double err_rate, double n_rate, const kc_synth_skew* skew,
                         void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* KC_API_H */
