/*
 * kman.h — C ABI of the MI355X (gfx950) k-mer extract / sort / join engine.
 *
 * The reference (ggirelli/kman, package kmermaid 1.0.0) is pure Python and has
 * no FFI of its own; its "operator API" is the class surface
 * FastaBatcher.do / Batch.sorted / Crawler.do_batch / KJoiner.join.  Every
 * entry point below replaces the arithmetic of one of those functions and is
 * what kman_amd/_native.py binds through ctypes:
 *
 *   kman_parse_fasta   SmartFastaParser.parse            kmermaid/parsers.py:86-128
 *                      + record name rule                 kmermaid/batcher.py:551
 *   kman_extract       Sequence.yield_kmers / kmerator    kmermaid/seq.py:285-359
 *                      + alphabet check / mkrc            kmermaid/seq.py:279,318,500-509
 *   kman_sort          Batch.sorted (stable, by .seq)     kmermaid/batch.py:156-168
 *                      + BatcherBase.write_all re-sort    kmermaid/batcher.py:133-153,392
 *   kman_sort_range    the same, by a prefix of the key bits
 *   kman_finish        Batch.sorted / Crawler.do_batch + join_* over prefix-sorted keys
 *                                                         batch.py:156-168, join.py:95-130,244-285
 *   kman_groups        the whole count / uniq chain of one stream:
 *                      yield_kmers -> Batch.sorted -> Crawler -> join_*
 *                                                         seq.py:285-328, batch.py:156-168,
 *                                                         join.py:63-130,244-285
 *   kman_rle_count     Crawler.do_batch + join_sequence_count
 *                                                         kmermaid/join.py:95-130,266-285
 *   kman_rle_uniq      Crawler.do_batch + join_unique     kmermaid/join.py:95-130,244-263
 *   kman_merge_runs    Crawler.do_records heapq.merge     kmermaid/join.py:63-93
 *   kman_format_*      the output writers                 kmermaid/join.py:262,284; seq.py:489-495
 *
 * Conventions
 *   - Plain C, no exceptions cross the boundary.  Every call returns 0 on
 *     success or a negative KMAN_E* code; kman_last_error() has the message.
 *   - Device buffers are raw device pointers obtained from kman_malloc and
 *     owned by the caller (freed with kman_free).  Host buffers are borrowed
 *     for the duration of the call.
 *   - One context per GPU and host thread; a context is not re-entrant.  All
 *     device work of a context runs in order on its own HIP stream.
 *   - Keys are k-mers packed 2 bits per base MSB-first (A=0 C=1 G=2 T=3), so
 *     numeric order of keys == the reference's Python str order of the
 *     upper-case sequences (for a fixed k <= 32).
 *   - "pos" payloads are (global base index << 1) | strand, where the global
 *     base index addresses the cleaned, concatenated sequence of all records
 *     (see kman_parse_fasta) and strand 1 means the '-' (reverse-complement)
 *     record of seq.py:274-282.
 */
#ifndef KMAN_H
#define KMAN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KMAN_ABI_VERSION 1

/* error codes */
#define KMAN_OK 0
#define KMAN_EINVAL (-1)   /* bad argument (maps to AssertionError like the reference) */
#define KMAN_EHIP (-2)     /* HIP runtime error */
#define KMAN_ENOMEM (-3)   /* device or host allocation failed */
#define KMAN_EFORMAT (-4)  /* input is not parsable FASTA (parsers.py:105-107) */
#define KMAN_ETIMEOUT (-5) /* a device-side wait exceeded its bound (engine bug) */
#define KMAN_ECOMM (-6)    /* RCCL error */
#define KMAN_ECAP (-7)     /* output capacity too small; *needed reports the size */
#define KMAN_EFALLBACK (-8) /* kman_groups: input outside the region path; use the general path */
#define KMAN_EPARTIAL (-9)  /* kman_dround_finish: some key ranges left out (kman_dround_failed) */

/* kman_extract flags */
#define KMAN_RC 1u          /* also emit reverse complements (kmer -r, seq.py:274-282) */
#define KMAN_WANT_POS 2u    /* also emit the pos payload (uniq / batch modes) */
#define KMAN_CANONICAL 4u   /* emit min(fwd, rc) instead (not in the reference) */
#define KMAN_MIXED 8u       /* with KMAN_CANONICAL: the canonical key through a fixed bijection of the
                             * 2k-bit keys (odd multiply, xorshift, odd multiply mod 2^2k), so the top
                             * bits are uniform; the multiset of counts is unchanged -- for abundance
                             * spectra (kman_groups, kman_dshard_*, kman_extract_marked / _range) */
#define KMAN_ONCE 16u       /* kman_dshard_hist / _extract: the shard is extracted ONCE for all key rounds
                             * (every window kept; the rounds' items in one buffer, round-major), so
                             * both use the tiles of a shard that one round takes (16 windows per
                             * thread, 8 with KMAN_RC); the same flags on both calls */
#define KMAN_ROOMY 32u      /* kman_dround_plan / _finish: pass-1 sub-regions planned at twice their
                             * expected fill (a genome's repeat families then fit, so regions its
                             * finish leaves out can be redone from pass 1's output, kman_dround_left);
                             * the same flags on both calls */
/* kman_extract: accumulate d_hist for the passes over bits [b, 2k) only
 * (the prefix passes of kman_split_bits); default b = 0, every bit */
#define KMAN_HIST_LO(b) (((uint32_t)(b) & 0x7fu) << 8)
#define KMAN_HIST_LO_OF(flags) (((flags) >> 8) & 0x7fu)

/* kman_finish modes */
#define KMAN_FINISH_SORT 0  /* full stable sort, in place          (batch.py:156-168) */
#define KMAN_FINISH_COUNT 1 /* (key, group size) per distinct key  (join.py:266-285) */
#define KMAN_FINISH_UNIQ 2  /* keys occurring once + payload       (join.py:244-263) */

typedef struct kman_ctx kman_ctx;

/* parse result (host struct) */
typedef struct {
    uint64_t n_bases;   /* cleaned sequence characters over all records */
    uint64_t n_records; /* header lines ('>' at a line start) */
} kman_parse_info;

/* ------------------------------------------------------------------ context */
int kman_abi_version(void);
int kman_device_count(int *n);
int kman_create(int device, kman_ctx **out);
void kman_destroy(kman_ctx *ctx);
const char *kman_last_error(const kman_ctx *ctx);
int kman_sync(kman_ctx *ctx);

/* ------------------------------------------------------------------- memory */
int kman_malloc(kman_ctx *ctx, void **dptr, size_t bytes);
int kman_free(kman_ctx *ctx, void *dptr);
/* free / total HBM of the context's device: the sizing of the key ranges of
 * a multi-batch join (kman_extract_range) */
int kman_mem_info(kman_ctx *ctx, size_t *free_bytes, size_t *total_bytes);
int kman_host_alloc(kman_ctx *ctx, void **hptr, size_t bytes); /* pinned */
int kman_host_free(kman_ctx *ctx, void *hptr);
int kman_memcpy_h2d(kman_ctx *ctx, void *dst, const void *src, size_t bytes);
int kman_memcpy_d2h(kman_ctx *ctx, void *dst, const void *src, size_t bytes);
int kman_memset(kman_ctx *ctx, void *dst, int value, size_t bytes);
/* Chunked uploads that overlap the context's work: kman_copy_h2d_async
 * enqueues a copy (from pinned memory for real overlap) on the context's copy
 * stream and marks event `slot` (0..3); kman_copy_wait makes the work stream
 * wait for that event; kman_copy_sync drains the copy stream.  The copy does
 * not wait for the work stream: a caller reusing a destination that queued
 * work still reads synchronises first (kman_sync). */
int kman_copy_h2d_async(kman_ctx *ctx, void *dst, const void *src, size_t bytes, int slot);
int kman_copy_wait(kman_ctx *ctx, int slot);
int kman_copy_sync(kman_ctx *ctx);
/* Downloads that overlap the context's work (formatted output text):
 * kman_copy_d2h_async queues a device -> host copy on the copy stream after
 * the work already queued (dst: pinned host memory, kman_host_alloc), marked
 * in d2h slot 0..3; kman_copy_d2h_wait blocks the calling host thread until
 * that copy is done. */
int kman_copy_d2h_async(kman_ctx *ctx, void *dst, const void *src, size_t bytes, int slot);
int kman_copy_d2h_wait(kman_ctx *ctx, int slot);

/* ------------------------------------------------------------------- timing
 * Optional per-kernel timing with HIP events recorded on the context's own
 * stream around every launch (bench.py's live roofline).  Tags: "parse",
 * "extract", "sort_hist", "sort_pass", "rle_count", "rle_uniq".
 * kman_timing_query synchronises and returns launches and summed ms. */
int kman_timing_enable(kman_ctx *ctx, int enable);
int kman_timing_query(kman_ctx *ctx, const char *tag, uint64_t *launches, double *total_ms);

/* ------------------------------------------------------------------- stages */

/* FASTA text -> cleaned base codes + record table  (parsers.py:86-128)
 *   d_text     n_bytes of FASTA text (uncompressed)
 *   d_codes    out, capacity >= n_bytes + 64: one byte per kept sequence char:
 *              bits 0-1 base (A/a=0 C/c=1 G/g=2 T/t=3), bit 2 set = not ACGT,
 *              bit 3 set = first char of a record.  64 pad bytes (value 4)
 *              follow the last code.
 *   d_rec_hdr  out, byte offset of each record's '>'
 *   d_rec_seq  out, global base index of each record's first char
 *   rec_cap    capacity of the two record arrays; KMAN_ECAP if exceeded
 * Returns KMAN_EFORMAT when no line starts with '>' (empty file included). */
int kman_parse_fasta(kman_ctx *ctx, const uint8_t *d_text, uint64_t n_bytes, uint8_t *d_codes,
                     uint64_t *d_rec_hdr, uint64_t *d_rec_seq, uint64_t rec_cap,
                     kman_parse_info *info);
/* One chunk of a FASTA parsed into d_codes from code_off on (chunked H2D
 * streams and byte-range shards, kman_amd/shard.py).  The chunk starts at a
 * line start; flags KMAN_PARSE_IN_RECORD: the chunk continues a record (its
 * leading lines are sequence lines of the record opened before it; it may
 * hold no header, or nothing at all).  d_rec_seq entries and the 64 pad bytes
 * are at code_off + the chunk's own indices; d_rec_hdr holds byte offsets
 * within the chunk.  d_text and d_codes 16-byte aligned (code_off need not
 * be). */
#define KMAN_PARSE_IN_RECORD 1u
int kman_parse_fasta_at(kman_ctx *ctx, const uint8_t *d_text, uint64_t n_bytes, uint32_t flags, uint8_t *d_codes,
                        uint64_t code_off, uint64_t *d_rec_hdr, uint64_t *d_rec_seq, uint64_t rec_cap,
                        kman_parse_info *info);

/* Number of k-mers kman_extract will emit (valid windows x (RC ? 2 : 1)). */
int kman_count_kmers(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k,
                     uint32_t flags, uint64_t *n_kmers);

/* base codes -> packed keys in stream order (seq.py:285-328), k in [2, 32].
 *   d_keys     out, capacity cap keys
 *   d_pos      out (flags & KMAN_WANT_POS), u32 if pos_bytes == 4 else u64
 *   d_hist     optional out (may be NULL): the radix-digit histograms that
 *              kman_sort would compute, for the pass plan of kman_sort_plan(2k)
 *              (npass x 256 u64, must be zeroed by the caller) */
int kman_extract(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k,
                 uint32_t flags, uint64_t *d_keys, void *d_pos, uint32_t pos_bytes, uint64_t cap,
                 uint64_t *d_hist, uint64_t *n_kmers);

/* kman_extract restricted to the keys in [key_lo, key_hi] (inclusive), in
 * stream order: one key range of a multi-batch join (inputs whose k-mers do
 * not fit the device at once are processed range by range; the ranges'
 * outputs concatenate to the global sorted output, join.py:63-130).  Keys of
 * the range past `cap` are counted, not written: KMAN_ECAP then.  Size the
 * ranges with kman_kmer_prefix_hist. */
int kman_extract_range(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                       uint64_t key_lo, uint64_t key_hi, uint64_t *d_keys, void *d_pos, uint32_t pos_bytes,
                       uint64_t cap, uint64_t *d_hist, uint64_t *n_kmers);
/* The same for the keys whose top map_bits bits p have d_map[p] == map_val
 * (d_map: 2^map_bits bytes): the key ranges a round left out
 * (kman_dround_failed), each destination's in one pass. */
int kman_extract_marked(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                        const uint8_t *d_map, uint32_t map_bits, uint32_t map_val, uint64_t *d_keys, void *d_pos,
                        uint32_t pos_bytes, uint64_t cap, uint64_t *n_kmers);
/* Histogram of the top 8 key bits of the stream (256 u64 into d_hist256) and
 * the k-mer count; flags: KMAN_RC (not KMAN_CANONICAL). */
int kman_kmer_prefix_hist(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                          uint64_t *d_hist256, uint64_t *n_kmers);

/* LSD radix sort plan for keys with key_bits significant bits:
 * npass digit passes of bits[i] bits each, starting at bit shift[i]. */
int kman_sort_plan(uint32_t key_bits, uint32_t *npass, uint32_t *shift, uint32_t *bits);

/* Stable LSD radix sort (onesweep, decoupled look-back) of n keys with an
 * optional payload (val_bytes 0, 4 or 8).  Ping-pongs between the two
 * buffers; *result_in_alt is set to 1 when the sorted data ended in the alt
 * buffers.  d_hist may be NULL (then computed) or the histogram filled by
 * kman_extract for the same key_bits.  Stability == the reference's Timsort
 * stability (batch.py:165). */
int kman_sort(kman_ctx *ctx, uint64_t *d_keys, uint64_t *d_keys_alt, void *d_vals, void *d_vals_alt,
              uint32_t val_bytes, uint64_t n, uint32_t key_bits, const uint64_t *d_hist,
              int *result_in_alt);

/* The same sort restricted to bits [lo_bit, hi_bit): a stable sort by those
 * bits only.  d_hist: NULL or kman_extract's with KMAN_HIST_LO(lo_bit). */
int kman_sort_plan_range(uint32_t lo_bit, uint32_t hi_bit, uint32_t *npass, uint32_t *shift,
                         uint32_t *bits);
int kman_sort_range(kman_ctx *ctx, uint64_t *d_keys, uint64_t *d_keys_alt, void *d_vals, void *d_vals_alt,
                    uint32_t val_bytes, uint64_t n, uint32_t lo_bit, uint32_t hi_bit, const uint64_t *d_hist,
                    int *result_in_alt);

/* Prefix-split sort: kman_sort_range over the top bits [lo_bit, key_bits)
 * (kman_split_bits picks lo_bit so that equal-prefix segments average <= 512
 * keys), then kman_finish completes the order of every segment in LDS and
 * emits in the same pass (Batch.sorted + Crawler.do_batch, batch.py:156-168,
 * join.py:95-130):
 *   SORT   d_keys / d_vals fully sorted in place (stable); *n_out = n
 *   COUNT  d_okeys[j], d_ovals[j] = group size (oval_bytes 4 | 8); d_vals unused
 *   UNIQ   d_okeys[j], d_ovals[j] = payload of keys that occur once
 *          (oval_bytes == val_bytes)
 * Input: keys stably sorted by bits [lo_bit, key_bits).  In COUNT / UNIQ mode
 * the input arrays are scratch afterwards (segments longer than a chunk's
 * staging area are sorted in place through d_*_alt-free temporary buffers). */
int kman_split_bits(uint64_t n, uint32_t key_bits, uint32_t *lo_bit);

/* kman_extract + kman_sort_range(lo_bit, 2k) in one call: the first prefix
 * pass is fused into the extraction (a histogram pre-pass over the codes, then
 * one kernel that rolls the windows and scatters them by digit 0), so the
 * keys are never written in stream order.  Same result as the two calls;
 * flags as kman_extract's (KMAN_CANONICAL, k > 25 or u64 pos run the two calls). */
int kman_extract_sorted(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                        uint32_t lo_bit, uint64_t *d_keys, uint64_t *d_keys_alt, void *d_pos, void *d_pos_alt,
                        uint32_t pos_bytes, uint64_t cap, uint64_t *n_kmers, int *result_in_alt);
int kman_finish(kman_ctx *ctx, uint64_t *d_keys, uint64_t *d_keys_alt, void *d_vals, void *d_vals_alt,
                uint32_t val_bytes, uint64_t n, uint32_t key_bits, uint32_t lo_bit, int mode,
                uint64_t *d_okeys, void *d_ovals, uint32_t oval_bytes, uint64_t *n_out);

/* Count / uniq of one k-mer stream straight from the base codes, through
 * padded regions of packed items (region.hip): extraction scattered by the
 * top 8 key bits, one pass per 8-bit bucket by the next bits, then one LDS
 * block per region sorts, groups and emits.  Replaces the chain
 * Sequence.yield_kmers -> Batch.sorted -> Crawler.do_records/do_batch ->
 * KJoiner.join_sequence_count | join_unique (seq.py:285-328,
 * batch.py:156-168, join.py:63-130,244-285) for one batch stream; same output
 * arrays as kman_extract_sorted + kman_finish(COUNT | UNIQ):
 *   COUNT  d_okeys[j], d_ovals[j] = group size (oval_bytes 4 | 8)
 *   UNIQ   d_okeys[j], d_ovals[j] = pos of the keys that occur once
 * in ascending key order; *n_kmers = k-mers extracted, *n_out = rows.
 * With KMAN_CANONICAL the keys are min(forward, reverse complement), one per
 * window.
 * kman_groups_plan gives the work-area size, or KMAN_EFALLBACK when the input
 * is outside the path (k > 25, too many k-mers for the region capacities).  kman_groups returns KMAN_EFALLBACK also when a region
 * overflowed (a strongly skewed prefix distribution); the outputs are then
 * undefined and the caller runs the general path.  d_okeys / d_ovals hold
 * up to n_bases x (RC ? 2 : 1) entries. */
int kman_groups_plan(uint64_t n_bases, uint32_t k, uint32_t flags, int mode, uint64_t *work_bytes);
int kman_groups(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags, int mode,
                void *d_work, uint64_t work_bytes, uint64_t *d_okeys, void *d_ovals, uint32_t oval_bytes,
                uint64_t *n_kmers, uint64_t *n_out);

/* kman_groups in three calls, so that its first pass (the extraction) runs
 * while the FASTA is still arriving (the reference reads and extracts one
 * record at a time, batcher.py:454-470 -> seq.py:285-328):
 *   kman_groups_begin    plans, clears the work area and opens the pass;
 *                        *n_tiles tiles, tile t reads codes
 *                        [t * tile_bases, (t + 1) * tile_bases + 64)
 *                        (*n_tiles = 0: the pass runs whole at the end)
 *   kman_groups_extract  extracts tiles up to tile_hi (exclusive) once their
 *                        codes are final; call in increasing tile_hi
 *   kman_groups_end      extracts the rest, then as kman_groups
 * Every call takes the arguments kman_groups takes (n_bases = the final
 * total); no other call of this ctx that uses look-back status words (the
 * general extraction, sorts, other kman_groups) may come in between.  The
 * result equals kman_groups'. */
int kman_groups_begin(kman_ctx *ctx, uint64_t n_bases, uint32_t k, uint32_t flags, int mode, void *d_work,
                      uint64_t work_bytes, uint32_t *n_tiles, uint64_t *tile_bases);
int kman_groups_extract(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                        int mode, void *d_work, uint64_t work_bytes, uint32_t tile_hi);
int kman_groups_end(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags, int mode,
                    void *d_work, uint64_t work_bytes, uint64_t *d_okeys, void *d_ovals, uint32_t oval_bytes,
                    uint64_t *n_kmers, uint64_t *n_out);

/* kman_groups across G ranks, in key rounds (one process per GPU over RCCL;
 * kman_amd/dist.py runs the collectives in between).  Rank q
 * holds one byte-range shard of ONE FASTA (its own bytes plus a (k-1)-base
 * halo, see kman_parse_fasta_at); every rank passes the same n_bases_q >=
 * every shard's n_bases (it fixes the pos bits of the packed 8-byte items).
 *   kman_dshard_plan     KMAN_OK, or KMAN_EFALLBACK outside the path (k > 25,
 *                        uniq pos bits + 2k - 8 > 64)
 *   kman_dshard_hist     exact item counts of the shard per (top-8-bit
 *                        bucket b, position segment s): hist[b * 64 + s]
 *                        (host copy of d_hist, 256 x 64 u32)
 *   (caller)             all-gather of the bucket totals; buckets cut into
 *                        G x R contiguous parts: rank q owns parts q*R ..
 *                        q*R+R-1, round r handles part q*R+r of every q
 *   kman_dshard_extract  one round's pass 0: the items of the buckets with
 *                        d_rtab[b * 64 + s] != ~0 written straight into
 *                        d_send, region (b, s) at d_rtab[b * 64 + s]
 *                        (destination-major, no padding, no gather)
 *   (caller)             one all-to-all of the items (kman_alltoallv, 8 B)
 *   kman_dround_plan     arena sizes of one round's finish on a rank
 *   kman_dround_finish   the received items of buckets [b_lo, b_lo + nb)
 *                        (source chunks in rank order, each in bucket order;
 *                        counts[src * nb + j] = items of bucket b_lo + j from
 *                        src) -> the round's count / uniq rows, ascending
 *                        (uniq pos u64 with the source rank in bits 56-63);
 *                        KMAN_EPARTIAL when regions overflowed (skewed
 *                        keys): their key ranges are left out (below).
 *                        d_a (>= a_bytes) may be the send buffer, d_b (>=
 *                        b_bytes) may be d_recv itself.
 * A rank's rounds emit its key range in order; the ranks' outputs in rank
 * order are the global output (Crawler.do_records / do_batch over all
 * batches, join.py:63-130). */
int kman_dshard_plan(uint64_t n_bases, uint64_t n_bases_q, uint32_t k, uint32_t flags, int mode);
int kman_dshard_hist(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint64_t n_bases_q, uint32_t k,
                     uint32_t flags, int mode, uint32_t *d_hist, uint32_t *hist);
int kman_dshard_extract(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint64_t n_bases_q, uint32_t k,
                        uint32_t flags, int mode, const uint32_t *d_hist, const uint64_t *d_rtab, uint64_t *d_send);
int kman_dround_plan(uint32_t k, uint32_t flags, int mode, uint32_t world, uint64_t n_bases_q, uint32_t nb,
                     const uint64_t *counts, uint64_t *a_bytes, uint64_t *b_bytes);
int kman_dround_finish(kman_ctx *ctx, const uint64_t *d_recv, uint32_t k, uint32_t flags, int mode, uint32_t world,
                       uint64_t n_bases_q, uint32_t b_lo, uint32_t nb, const uint64_t *counts, void *d_a,
                       uint64_t a_bytes, void *d_b, uint64_t b_bytes, uint64_t *d_okeys, void *d_ovals,
                       uint32_t oval_bytes, uint64_t *n_out);
/* After kman_dround_finish returned KMAN_EPARTIAL: regions that overflowed a
 * capacity (a key repeated far beyond its region's share) emitted nothing,
 * the other *n_out rows are in place in key order.  kman_dround_failed gives
 * the left-out key ranges as [lo, hi] pairs (2 u64 each, ascending, merged;
 * *n = ranges; NULL ranges: count only) for the caller to redo through
 * kman_extract_marked + kman_sort_range + kman_finish and merge in
 * (kman_merge_runs). */
int kman_dround_failed(kman_ctx *ctx, uint64_t *ranges, uint64_t cap, uint64_t *n);
/* Heavy keys of the last kman_dround_finish (*n; 0 when none or off): keys
 * that every S-th received item's sample saw at least twice (the most often
 * sampled, at most 256 per bucket of the round, held in the pass's LDS while
 * a chain of the bucket runs) are counted apart in its pass 1 -- count mode
 * keeps one copy per pass-1 chain and adds the others to the key's row after
 * the finish, uniq mode drops them all (they occur more than once) -- so a
 * repeat with 10^5 copies does not overflow its regions.  KMAN_HEAVY=0 turns
 * it off, KMAN_HEAVY=1 applies it to rounds of any size (default: >= 2^20
 * items).  Not in the reference: the rows are the same either way. */
int kman_dround_heavy(kman_ctx *ctx, uint32_t *n);
/* After kman_dround_finish (before its arena A is reused): the items of the
 * regions it left out, gathered from its pass-1 output instead of
 * re-extracted from the codes (kman_extract_marked) -- full keys in d_keys
 * and, uniq, the pos its finish would have emitted in d_pos; *n = items
 * (NULL d_keys: count only; cap = room in d_keys / d_pos).  KMAN_EFALLBACK
 * when its pass 1 itself overflowed (its output lacks items): then the
 * marked extraction.  The items' sort + run-length rows equal the left-out
 * regions' rows once kman_dround_heavy_fix has added the heavy keys' dropped
 * copies (count mode).  Not in the reference. */
int kman_dround_left(kman_ctx *ctx, uint64_t *d_keys, uint64_t *d_pos, uint64_t cap, uint64_t *n);
/* Adds the last kman_dround_finish's heavy keys' dropped copies to the rows
 * (d_keys sorted) that hold them: for rows built from kman_dround_left's
 * items (count mode; uniq rows and rows recounted from the codes need none). */
int kman_dround_heavy_fix(kman_ctx *ctx, const uint64_t *d_keys, void *d_vals, uint32_t val_bytes, uint64_t n);

/* Abundance spectrum of a count output (BASELINE config 5; not
 * in the reference): d_hist[c] = number of distinct k-mers seen c times, the
 * last bin collecting every count >= nbins - 1 (bin 0 stays 0).  With
 * KMAN_CANONICAL counts (kman_groups) this is the canonical k-mer spectrum;
 * for odd k those counts equal the `kmer count -r` rows with key <= rc(key)
 * (the reference's -r emits both strands, seq.py:274-282).  d_counts 16-byte aligned. */
int kman_count_hist(kman_ctx *ctx, const void *d_counts, uint32_t count_bytes, uint64_t n, uint64_t *d_hist,
                    uint32_t nbins);

/* k in 33..64 (Sequence.yield_kmers has no k limit, seq.py:285-328): keys
 * as word pairs, hi = the first k - 32 bases (2(k-32) bits), lo = the last 32
 * bases, both 2 bits per base MSB-first, so (hi, lo) in lexicographic order is
 * the reference's str order.
 *   kman_extract_wide  keys (+ pos) in stream order; d_hi = d_lo = NULL only
 *                      counts (*n_kmers); flags KMAN_RC | KMAN_CANONICAL |
 *                      KMAN_WANT_POS as kman_extract
 *   kman_iota_u64      v[i] = i
 *   kman_gather        dst[i] = src[idx[i]] (4 or 8 byte elements)
 *   kman_rle_wide      count / uniq of (hi, lo) pairs sorted lexicographically
 *                      (mode KMAN_FINISH_COUNT: d_ovals = group sizes; UNIQ:
 *                      the pairs of groups of one with their d_vals payload)
 * The sort is two stable kman_sort passes: by lo with an index payload, then
 * by the gathered hi (an LSD sort over 2k bits); the host writers
 * kman_format_*_wide print the pairs. */
int kman_extract_wide(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                      uint64_t *d_hi, uint64_t *d_lo, void *d_pos, uint32_t pos_bytes, uint64_t cap,
                      uint64_t *n_kmers);
int kman_iota_u64(kman_ctx *ctx, uint64_t *d_v, uint64_t n);
int kman_gather(kman_ctx *ctx, const void *d_src, const uint64_t *d_idx, uint64_t n, void *d_dst, uint32_t elem_bytes);
int kman_rle_wide(kman_ctx *ctx, int mode, const uint64_t *d_hi, const uint64_t *d_lo, const void *d_vals,
                  uint32_t val_bytes, uint64_t n, uint64_t *d_ohi, uint64_t *d_olo, void *d_ovals, uint64_t *n_out);

/* Any k >= 2 (the reference has no k limit: Sequence.yield_kmers,
 * seq.py:285-328; FastaBatcher.do asserts only k > 1, batcher.py:477-478):
 * a k-mer as W = ceil(k / 32) words, MSB-first -- word 0 the first
 * k - 32 (W - 1) bases, words 1 .. W-1 32 bases each -- so (w_0 .. w_{W-1})
 * in lexicographic order is the reference's str order (Batch.sorted,
 * batch.py:156-168).  Word-major planes: word j of item i at
 * d_words[j * stride + i] (W = 2 is kman_extract_wide's (hi, lo)).
 *   kman_extract_words  keys (+ pos, (global base << 1) | strand) of the valid
 *                       windows in stream order (records, positions, + then
 *                       - with KMAN_RC; one min(fwd, rc) key per window with
 *                       KMAN_CANONICAL); d_words = d_pos = NULL only counts;
 *                       KMAN_ECAP (with *n_out) when more than cap
 *   kman_rle_words      count / uniq of sorted word keys (Crawler.do_batch +
 *                       join_sequence_count / join_unique, join.py:95-130,
 *                       244-285): KMAN_FINISH_COUNT -> d_ovals = group sizes;
 *                       UNIQ -> the keys of groups of one with their d_vals
 *   kman_batch_tags     d_tags[i] = (start + d_perm[i]) / per_batch: the batch
 *                       of every item of a permutation of stream range
 *                       [start, ..) (Batch.sorted per batch, batch.py:156-168)
 * The sort is LSD over the planes: stable kman_sort passes with an index
 * payload and kman_gather (kman_amd/engine.py sort_words). */
int kman_extract_words(kman_ctx *ctx, const uint8_t *d_codes, uint64_t n_bases, uint32_t k, uint32_t flags,
                       uint64_t *d_words, uint64_t stride, void *d_pos, uint32_t pos_bytes, uint64_t cap,
                       uint64_t *n_out);
int kman_rle_words(kman_ctx *ctx, int mode, const uint64_t *d_words, uint32_t W, uint64_t stride, const void *d_vals,
                   uint32_t val_bytes, uint64_t n, uint64_t *d_owords, uint64_t ostride, void *d_ovals,
                   uint32_t oval_bytes, uint64_t *n_out);
int kman_batch_tags(kman_ctx *ctx, const uint64_t *d_perm, uint64_t n, uint64_t start, uint64_t per_batch,
                    uint64_t *d_tags);

/* Run-length count of sorted keys (join.py:95-130 + 266-285):
 * d_ukeys[j], d_counts[j] (u32 if count_bytes == 4 else u64). */
int kman_rle_count(kman_ctx *ctx, const uint64_t *d_keys, uint64_t n, uint64_t *d_ukeys,
                   void *d_counts, uint32_t count_bytes, uint64_t *n_unique);

/* n-way merge of runs each sorted by key (Crawler.do_records' heapq.merge
 * over sorted batches, kmermaid/join.py:63-93): a tree of stable merge-path
 * 2-way merges in run order, so equal keys keep run order, then in-run order.
 * d_okeys / d_ovals get the merged total; d_tmp_* (same size) is scratch
 * (unused for <= 2 runs).  val_bytes 0 (keys only), 4 or 8.
 * kman_count_descents: number of i with keys[i] < keys[i-1] (0 = sorted). */
typedef struct {
    const uint64_t *keys;
    const void *vals;
    uint64_t n;
} kman_run;
int kman_merge_runs(kman_ctx *ctx, const kman_run *runs, int nruns, uint32_t val_bytes, uint64_t *d_okeys,
                    void *d_ovals, uint64_t *d_tmp_keys, void *d_tmp_vals);
int kman_count_descents(kman_ctx *ctx, const uint64_t *d_keys, uint64_t n, uint64_t *descents);
/* kman_row_digest: a checksum of n result rows (keys + 0 / 4 / 8-byte values)
 * for comparing two joins' outputs without moving them to the host (the
 * at-size tests): out4 = {sum, xor} of h_i = mix(key_i ^ mix(val_i + (first +
 * i) * 0x9E3779B97F4A7C15)) (mix = the murmur3 finaliser), the sum of the
 * values, and the number of i >= 1 with keys[i] <= keys[i-1].  Sums are mod
 * 2^64; slices [a, b) digested with first = a combine by sum / xor / sum. */
int kman_row_digest(kman_ctx *ctx, const uint64_t *d_keys, const void *d_vals, uint32_t val_bytes, uint64_t n,
                    uint64_t first_index, uint64_t *out4);

/* Abundance vectors, KJoiner VEC_COUNT / VEC_COUNT_MASKED (join.py:288-335 ->
 * AbundanceVector.add_count, abundance.py:103-130; the reference's base-class
 * call raises NotImplementedError, so these are its evident semantics): over
 * a key-sorted, stream-stable array with pos payloads ((window << 1) | strand,
 * tagged with the source in bits 56-63 when `tagged`), write d_vec[index] =
 * the size of the item's key run (masked = 0), or (masked = 1) the run's
 * items in other records, only when the run spans several records.  index =
 * pos, or src_base[pos >> 56] + (pos & (2^56 - 1)) when tagged.  Masked:
 * rec_start (nrec ascending, index space) and rec_id (the record identity,
 * one per distinct name) give each item's record.  d_vec (u32) is zeroed by
 * the caller; entries never written stay 0. */
int kman_vec_fill(kman_ctx *ctx, const uint64_t *d_keys, const void *d_pos, uint32_t pos_bytes, uint64_t n,
                  int masked, const uint64_t *d_src_base, uint32_t tagged, const uint64_t *d_rec_start,
                  const uint32_t *d_rec_id, uint64_t nrec, uint32_t *d_vec);
/* Host: one vector as text, "%d\n" per entry v[0], v[stride], .. (n entries;
 * AbundanceVector.write_to, abundance.py:151-168); out NULL: size only. */
int kman_format_vector(const uint32_t *v, uint64_t n, uint64_t stride, char *out, size_t cap, size_t *used,
                       int threads);

/* Keys that occur exactly once, with their payload (join.py:244-263). */
int kman_rle_uniq(kman_ctx *ctx, const uint64_t *d_keys, const void *d_vals, uint32_t val_bytes,
                  uint64_t n, uint64_t *d_okeys, void *d_ovals, uint64_t *n_out);

/* ------------------------------------------------------------ multi-GPU
 * One process per GPU over RCCL (xGMI).  The reference has no collective
 * (joblib pools over temp files); this is the single exchange step that
 * splits the global join by prefix range.
 *   kman_comm_unique_id  rank 0 creates the 128-byte id, the launcher shares it
 *   kman_comm_init       ncclCommInitRank on the context's device
 *   kman_comm_count      the ranks and this rank as the communicator counts
 *                        them (ncclCommCount / ncclCommUserRank)
 *   kman_prefix_hist     d_hist[(key >> shift) & (2^bits - 1)] += 1 (bits <= 14)
 *   kman_allreduce_u64   in-place sum (histograms)
 *   kman_allgather_u64   per-rank counts
 *   kman_alltoallv       grouped send/recv of contiguous per-destination runs
 *   kman_partition       stable partition of keys (+ vals) into nbuckets
 *                        destinations, bucket = d_lut[key >> lut_shift]; one
 *                        onesweep pass; bucket_counts is a host array */
int kman_comm_unique_id(uint8_t *out128);
int kman_comm_init(kman_ctx *ctx, const uint8_t *id128, int nranks, int rank);
int kman_comm_count(kman_ctx *ctx, int *nranks, int *rank);
int kman_comm_destroy(kman_ctx *ctx);
int kman_prefix_hist(kman_ctx *ctx, const uint64_t *d_keys, uint64_t n, uint32_t shift, uint32_t bits,
                     uint64_t *d_hist);
int kman_allreduce_u64(kman_ctx *ctx, uint64_t *d_buf, uint64_t n);
int kman_allgather_u64(kman_ctx *ctx, const uint64_t *d_send, uint64_t *d_recv, uint64_t n);
int kman_alltoallv(kman_ctx *ctx, const void *d_send, const uint64_t *send_counts, const uint64_t *send_offsets,
                   void *d_recv, const uint64_t *recv_counts, const uint64_t *recv_offsets, uint32_t elem_bytes);
/* The same on the context's communication stream, ordered after the work
 * queued so far on its compute stream; completion recorded in event `slot`
 * (0..7).  kman_comm_wait makes the compute stream wait for it: an exchange
 * overlaps the compute on the parts already received (DistPipeline's
 * overlapped rounds). */
int kman_alltoallv_async(kman_ctx *ctx, const void *d_send, const uint64_t *send_counts,
                         const uint64_t *send_offsets, void *d_recv, const uint64_t *recv_counts,
                         const uint64_t *recv_offsets, uint32_t elem_bytes, int slot);
int kman_comm_wait(kman_ctx *ctx, int slot);
int kman_partition(kman_ctx *ctx, const uint64_t *d_keys, uint64_t *d_keys_out, const void *d_vals,
                   void *d_vals_out, uint32_t val_bytes, uint64_t n, const uint8_t *d_lut, uint32_t lut_shift,
                   uint32_t nbuckets, const uint64_t *bucket_counts);

/* ------------------------------------------------------------ helpers
 * kman_tag_batches: keys[i] |= ((first_index + i) / batch_size) << key_bits,
 *   so one stable kman_sort over key_bits + tag bits sorts every stream chunk
 *   of batch_size k-mers on its own (BatcherBase.new_batch, batcher.py:118-131,
 *   then Batch.sorted per batch).  KMAN_EINVAL if the tag does not fit.
 * kman_or_u64 / kman_widen_u32: payload tagging (multi-source joins). */
int kman_tag_batches(kman_ctx *ctx, uint64_t *d_keys, uint64_t n, uint32_t key_bits, uint64_t first_index,
                     uint64_t batch_size);
int kman_or_u64(kman_ctx *ctx, uint64_t *d_v, uint64_t n, uint64_t value);
int kman_widen_u32(kman_ctx *ctx, const uint32_t *d_in, uint64_t *d_out, uint64_t n, uint64_t value);
int kman_memcpy_d2d(kman_ctx *ctx, void *dst, const void *src, size_t bytes);
/* kman_rebase_pos: uniq pos tagged with their source shard (bits 56-63) ->
 *   global pos: (pos & (2^56 - 1)) + (offsets[source] << 1), offsets = the
 *   global base index of each shard's first base (host array, nsrc <= 256).
 * kman_synth_fasta: bytes [byte_lo, byte_lo + n_bytes) of the synthetic
 *   benchmark FASTA into d_out (16-byte aligned): records r = 0.. with header
 *   ">syn<r>\n" at byte rec_tab[3r], first base index rec_tab[3r + 1] and
 *   rec_tab[3r + 2] bases in lines of `line` bases + "\n"; base i of the file
 *   = "ACGT"[splitmix64(seed * 0xD1B54A32D192ED03 + i) >> 62] (the same
 *   generator as tests/golden/inputs.py synth_np). */
int kman_rebase_pos(kman_ctx *ctx, uint64_t *d_pos, uint64_t n, const uint64_t *offsets, uint32_t nsrc);
int kman_synth_fasta(kman_ctx *ctx, uint8_t *d_out, uint64_t byte_lo, uint64_t n_bytes, uint64_t seed,
                     const uint64_t *rec_tab, uint32_t n_records, uint32_t line);

/* ------------------------------------------------------------- formatting
 * Host-side writers that produce the reference's exact bytes.  They run on
 * host threads over host copies of the device results.
 *   names      concatenated record names, name r at names[name_off[r] .. name_off[r+1])
 *   rec_seq    host copy of d_rec_seq (sorted ascending)
 * Each returns the number of bytes written to out (<= cap) in *used, or
 * KMAN_ECAP with the required size in *used. */
int kman_format_count(const uint64_t *ukeys, const void *counts, uint32_t count_bytes, uint64_t n,
                      uint32_t k, char *out, size_t cap, size_t *used, int threads);
int kman_format_uniq(const uint64_t *keys, const void *pos, uint32_t pos_bytes, uint64_t n,
                     uint32_t k, const char *names, const uint64_t *name_off,
                     const uint64_t *rec_seq, uint64_t n_records, char *out, size_t cap,
                     size_t *used, int threads);

/* uniq rows of a multi-source join (several FASTA inputs and reloaded batch
 * files, join.py:63-93 + 244-263): pos are u64 global base indices over one
 * merged record table; rec_kind[r] 0 = a FASTA record (header
 * name:start-end:strand), 1 = a batch-file record printed by its title. */
int kman_format_uniq_mixed(const uint64_t *keys, const uint64_t *pos, uint64_t n, uint32_t k, const char *names,
                           const uint64_t *name_off, const uint64_t *rec_seq, const uint8_t *rec_kind,
                           uint64_t n_records, char *out, size_t cap, size_t *used, int threads);
int kman_format_count_wide(const uint64_t *hi, const uint64_t *lo, const void *counts, uint32_t count_bytes,
                           uint64_t n, uint32_t k, char *out, size_t cap, size_t *used, int threads);
/* any k >= 2 over W word planes (kman_extract_words layout, row i's word j at
 * words[j * stride + i]) */
int kman_format_count_words(const uint64_t *words, uint64_t stride, const void *counts, uint32_t count_bytes,
                            uint64_t n, uint32_t k, char *out, size_t cap, size_t *used, int threads);
int kman_format_uniq_words(const uint64_t *words, uint64_t stride, const void *pos, uint32_t pos_bytes, uint64_t n,
                           uint32_t k, const char *names, const uint64_t *name_off, const uint64_t *rec_seq,
                           uint64_t n_records, char *out, size_t cap, size_t *used, int threads);
int kman_format_uniq_mixed_words(const uint64_t *words, uint64_t stride, const uint64_t *pos, uint64_t n, uint32_t k,
                                 const char *names, const uint64_t *name_off, const uint64_t *rec_seq,
                                 const uint8_t *rec_kind, uint64_t n_records, char *out, size_t cap, size_t *used,
                                 int threads);
int kman_format_uniq_wide(const uint64_t *hi, const uint64_t *lo, const void *pos, uint32_t pos_bytes, uint64_t n,
                          uint32_t k, const char *names, const uint64_t *name_off, const uint64_t *rec_seq,
                          uint64_t n_records, char *out, size_t cap, size_t *used, int threads);

/* The same writers on the device: the output text is built in
 * HBM (d_out, 16-byte aligned) from device-resident results, so only the text
 * crosses PCIe.  Byte-identical to kman_format_count / kman_format_uniq.
 * *used = the text size; KMAN_ECAP when it exceeds cap (nothing past cap is
 * written; d_out = NULL sizes only).  The rows are independent: a slice of
 * the result arrays formats to the matching slice of the text. */
int kman_format_count_dev(kman_ctx *ctx, const uint64_t *d_ukeys, const void *d_counts, uint32_t count_bytes,
                          uint64_t n, uint32_t k, char *d_out, size_t cap, size_t *used);
int kman_format_uniq_dev(kman_ctx *ctx, const uint64_t *d_keys, const void *d_pos, uint32_t pos_bytes, uint64_t n,
                         uint32_t k, const char *d_names, const uint64_t *d_name_off, const uint64_t *d_rec_seq,
                         uint64_t n_records, char *d_out, size_t cap, size_t *used);
/* k in 33..64: the same writers over word-pair keys (kman_extract_wide). */
int kman_format_count_wide_dev(kman_ctx *ctx, const uint64_t *d_hi, const uint64_t *d_lo, const void *d_counts,
                               uint32_t count_bytes, uint64_t n, uint32_t k, char *d_out, size_t cap, size_t *used);
int kman_format_uniq_wide_dev(kman_ctx *ctx, const uint64_t *d_hi, const uint64_t *d_lo, const void *d_pos,
                              uint32_t pos_bytes, uint64_t n, uint32_t k, const char *d_names,
                              const uint64_t *d_name_off, const uint64_t *d_rec_seq, uint64_t n_records, char *d_out,
                              size_t cap, size_t *used);

/* any k >= 2: the device writers over W word planes */
int kman_format_count_words_dev(kman_ctx *ctx, const uint64_t *d_words, uint64_t stride, const void *d_counts,
                                uint32_t count_bytes, uint64_t n, uint32_t k, char *d_out, size_t cap, size_t *used);
int kman_format_uniq_words_dev(kman_ctx *ctx, const uint64_t *d_words, uint64_t stride, const void *d_pos,
                               uint32_t pos_bytes, uint64_t n, uint32_t k, const char *d_names,
                               const uint64_t *d_name_off, const uint64_t *d_rec_seq, uint64_t n_records,
                               char *d_out, size_t cap, size_t *used);

#ifdef __cplusplus
}
#endif
#endif /* KMAN_H */
