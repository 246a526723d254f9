/* seqalib_hip.h — C ABI of the MI355X (gfx950) pairwise-alignment engine (libseqalib_hip.so).
 *
 * This is the drop-in boundary for the reference's DP hot path (przemektmalon/SeqALib):
 *   SequenceAligner::getAlignment (include/SequenceAlignment.h:153) as implemented by
 *     SmithWatermanSA::getAlignment   (include/SASmithWaterman.h:358-366)
 *     NeedlemanWunschSA::getAlignment (include/SANeedlemanWunsch.h:256-264)
 *     LocalGotohSA::getAlignment      (include/SALocalGotoh.h:518-526)
 *     GlobalGotohSA::getAlignment     (include/SAGlobalGotoh.h:450-459)
 * i.e. cacheAllMatches -> computeScoreMatrix -> buildResult, batched over independent pairs.
 * The header-only C++ API in include/seqalib/ (same class names and templates as the
 * reference) sits on top of this ABI; forceGlobal and the AlignedSequence list are built on the
 * host from the op stream returned here.
 *
 * Conventions: plain pointers and sizes, no C++ or torch types.  Every function returns an int
 * status (SA_OK = 0, negative on error) and never throws; sa_last_error() explains the last
 * failure on a context.  A context is bound to one device and must be used from one host thread
 * at a time (one context per GPU for multi-GPU work).
 */
#ifndef SEQALIB_HIP_H
#define SEQALIB_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SA_ABI_VERSION 1

/* Algorithms on the path. */
enum {
    SA_SW = 0,            /* SmithWatermanSA   — linear gap, local  (SASmithWaterman.h)   */
    SA_NW = 1,            /* NeedlemanWunschSA — linear gap, global (SANeedlemanWunsch.h) */
    SA_LOCAL_GOTOH = 2,   /* LocalGotohSA      — affine gap, local  (SALocalGotoh.h)      */
    SA_GLOBAL_GOTOH = 3,  /* GlobalGotohSA     — affine gap, global (SAGlobalGotoh.h)     */
    SA_HIRSCHBERG = 4,    /* HirschbergSA      — linear gap, global, linear space (SAHirschberg.h):
                             the reference's own split/tie rules, not just an optimal alignment;
                             score = NW H[m][n]; ops in traceback order like NW */
    SA_MYERS_MILLER = 5   /* MyersMillerSA     — affine gap, global, linear space (SAMyersMiller.h):
                             the reference's own midpoint/tie rules and base cases; reads
                             gap_open/gap_extend/match/mismatch/allow_mismatch; score = the top
                             call's optimum (the reference exposes none); ops like NW */
};

/* Status codes. */
enum {
    SA_OK = 0,
    SA_ERR_ARG = -1,          /* bad argument (null pointer, bad algo, inconsistent sizes)  */
    SA_ERR_HIP = -2,          /* HIP runtime error (no device, launch failure, ...)          */
    SA_ERR_NOMEM = -3,        /* device or host allocation failed                            */
    SA_ERR_CAPACITY = -4,     /* caller's output buffer (ops) too small                      */
    SA_ERR_UNSUPPORTED = -5   /* input outside what the engine supports (e.g. length >= 2^24) */
};

/* Per-pair result flags (sa_result.flags). */
enum {
    SA_FLAG_DIVERGED = 1,     /* the reference's traceback would never terminate here
                                 (only reachable with scorings whose gap terms are >= 0) */
    SA_FLAG_BAD_SHAPE = 2,    /* device API: pair longer than the max_m/max_n it was given */
    SA_FLAG_SIZE_HACK = 4,    /* LocalGotoh pair replaced by NW (SALocalGotoh.h:484-488)   */
    SA_FLAG_TIMEOUT = 8,      /* internal, never returned: a multi-workgroup (SPLIT) band's
                                 bounded wait for the band above it expired; the same call
                                 re-runs such pairs on the single-workgroup plan         */
    SA_FLAG_RECOVERED = 16    /* informational: a consistency guard of the band-parallel
                                 traceback fired and the pair was re-walked serially; the
                                 result is exact                                          */
};

/* ScoringSystem (include/SequenceAlignment.h:82-131).  Which fields are meaningful depends on
 * the constructor the caller used: linear algorithms read gap/match/mismatch/allow_mismatch,
 * affine algorithms read gap_open/gap_extend/match/mismatch/allow_mismatch.  For the 2-argument
 * form (Gap, Match) the reference sets Mismatch = INT_MIN and AllowMismatch = false. */
typedef struct {
    int32_t gap, match, mismatch, gap_open, gap_extend, allow_mismatch;
} sa_scoring;

/* One pair's result.
 *   score   SW/LocalGotoh: the maximum cell score (the reference's MaxScore);
 *           NW/GlobalGotoh: H[m][n] (M[m][n]).  SW on an empty input: INT32_MIN.
 *   end_i, end_j     SW/LocalGotoh: (MaxRow, MaxCol) — the last row-major cell holding the max;
 *                    NW/GlobalGotoh: (m, n).
 *   start_i, start_j where the traceback stopped (the forceGlobal idx1/idx2 for local modes).
 *   nops    number of ops written for this pair (traceback order, see below).
 * The ops of pair p live at ops + sa_ops_offset(p) where
 *   sa_ops_offset(p) = seq1_off[p] + seq2_off[p] + p   (room for m + n + 1 ops per pair). */
typedef struct {
    int32_t score;
    int32_t end_i, end_j;
    int32_t start_i, start_j;
    uint32_t nops;
    uint32_t flags;
    uint32_t reserved;
} sa_result;

/* Op codes, in traceback order (the order the reference's buildResult push_front()s them):
 *   'M' diagonal, match fn true       -> Entry(Seq1[i-1], Seq2[j-1], true),  i--, j--
 *   'S' diagonal, match fn false      -> Entry(Seq1[i-1], Seq2[j-1], false), i--, j--
 *   'U' up                            -> Entry(Seq1[i-1], Blank, false),     i--
 *   'L' left                          -> Entry(Blank, Seq2[j-1], false),     j--
 *   'X' diagonal, !AllowMismatch, no match -> Entry(Seq1[i-1],Blank) then Entry(Blank,Seq2[j-1])
 *   'u' / 'l' LocalGotoh gap-open whose score is <= 0: the entry of 'U' / 'L' without moving,
 *       then stop (SALocalGotoh.h:395-400 and :451-456). */

typedef struct sa_ctx sa_ctx;

/* Library / device discovery. */
int sa_version(void);
int sa_device_count(int* count);
const char* sa_status_string(int status);

/* Context lifetime.  sa_create binds to `device` (HIP ordinal) and allocates nothing large;
 * the device workspace grows on demand and is kept until sa_destroy / sa_trim. */
int sa_create(int device, sa_ctx** out);
void sa_destroy(sa_ctx* ctx);
const char* sa_last_error(const sa_ctx* ctx);
int sa_set_workspace_limit(sa_ctx* ctx, uint64_t bytes);   /* 0 = automatic (80% of free HBM) */
int sa_trim(sa_ctx* ctx);                                   /* free the cached workspace */

/* Cross-call pipeline of the device API (off by default).  When enabled, consecutive
 * sa_align_batch_device calls overlap: call k's traceback runs on an internal stream while call
 * k+1's fill runs on another, with SA_PIPELINE_DEPTH workspace slots (that many times the HBM).
 * A call is ordered after work
 * already enqueued on the caller's stream, but the caller's stream is NOT ordered after the
 * call's results: wait with sa_wait(ctx) (or a device-wide synchronize) before reading
 * d_results / d_ops, and give any SA_PIPELINE_DEPTH consecutive calls distinct output buffers.
 * Disabling waits for pipelined work.  The host API (sa_align_batch) never pipelines. */
#define SA_PIPELINE_DEPTH 2
int sa_set_pipeline(sa_ctx* ctx, int enable);
int sa_wait(sa_ctx* ctx);

/* Host-buffer batch API (used by the C++ drop-in headers).
 * seq1/seq2: concatenated symbol bytes; seq*_off: npairs+1 offsets (seq*_off[0] = 0).
 * match_lut: NULL for byte equality (the reference's `equal<char>` / nullptr match fn), or a
 *   256x256 table, match_lut[a*256 + b] != 0 iff match(a, b).
 * results: npairs entries.  ops: buffer of ops_cap bytes, pair p's ops at sa_ops_offset(p), so
 *   ops_cap >= seq1_off[npairs] + seq2_off[npairs] + npairs.
 * LocalGotoh pairs of the three sizes in SALocalGotoh.h:484-488 are aligned with NW, as the
 * reference does (flag SA_FLAG_SIZE_HACK).  Blocking; returns when results are on the host. */
int sa_align_batch(sa_ctx* ctx, int algo, const sa_scoring* scoring,
                   const uint8_t* seq1, const uint64_t* seq1_off,
                   const uint8_t* seq2, const uint64_t* seq2_off, uint32_t npairs,
                   const uint8_t* match_lut, sa_result* results, uint8_t* ops, uint64_t ops_cap);

/* sa_align_batch in `chunks` contiguous pair ranges of near-equal sum of m*n (0: one, or
 * $SEQALIB_HOST_CHUNKS), pipelined on the device (chunk g's traceback beside chunk g+1's fill), and
 * cb(user, pair_begin, pair_end) called on the calling thread as soon as a range's results and op
 * streams are in the caller's buffers -- so a caller can post-process chunk g (the C++ drop-in
 * builds its AlignedSequence lists) while later chunks are still on the GPU.  cb may be NULL.
 * LocalGotoh reports the whole batch once at the end; Hirschberg / Myers-Miller run as one chunk. */
typedef void (*sa_chunk_cb)(void* user, uint32_t pair_begin, uint32_t pair_end);
int sa_align_batch_cb(sa_ctx* ctx, int algo, const sa_scoring* scoring,
                      const uint8_t* seq1, const uint64_t* seq1_off,
                      const uint8_t* seq2, const uint64_t* seq2_off, uint32_t npairs,
                      const uint8_t* match_lut, sa_result* results, uint8_t* ops, uint64_t ops_cap,
                      uint32_t chunks, sa_chunk_cb cb, void* user);

/* Generic-Ty batch API (any symbol type, any number of distinct symbols: the path the C++
 * drop-in takes when a batch has more than 256 distinct symbols).  Instead of symbols the caller
 * passes each pair's match matrix -- the reference's cacheAllMatches (e.g. SASmithWaterman.h:
 * 20-45) packed to bits: pair p's bitmap starts at word bits_off[p] of `match_bits`, row-major,
 * ceil(n/32) 32-bit words per row, bit (j % 32) of word [i * ceil(n/32) + j / 32] =
 * match(Seq1[i], Seq2[j]).  seq*_off are the npairs+1 length offsets of the sequences (they
 * size the ops as in sa_align_batch); bits_off has npairs+1 entries.  SW, NW, LocalGotoh (with
 * the size hack) and GlobalGotoh; results and ops exactly as sa_align_batch.  Blocking. */
int sa_align_batch_bits(sa_ctx* ctx, int algo, const sa_scoring* scoring,
                        const uint64_t* seq1_off, const uint64_t* seq2_off, uint32_t npairs,
                        const uint32_t* match_bits, const uint64_t* bits_off,
                        sa_result* results, uint8_t* ops, uint64_t ops_cap);

/* Several GPUs of one node behind one handle.  sa_multi_create opens one persistent context per
 * listed device (a device may be listed twice).  sa_multi_align_batch has exactly the contract of
 * sa_align_batch: the batch is cut into contiguous pair ranges of near-equal sum of m*n, one per
 * context, aligned concurrently (one host thread each, no collective), and every range writes its
 * results and op streams in place in the caller's buffers. */
typedef struct sa_multi sa_multi;
int sa_multi_create(const int* devices, int ndevices, sa_multi** out);
void sa_multi_destroy(sa_multi* multi);
const char* sa_multi_last_error(const sa_multi* multi);
int sa_multi_align_batch(sa_multi* multi, int algo, const sa_scoring* scoring,
                         const uint8_t* seq1, const uint64_t* seq1_off,
                         const uint8_t* seq2, const uint64_t* seq2_off, uint32_t npairs,
                         const uint8_t* match_lut, sa_result* results, uint8_t* ops, uint64_t ops_cap);

/* Device-resident batch API: every pointer is device memory (HBM) and the work is enqueued on
 * `stream` (a hipStream_t; NULL = the context's own stream).  Asynchronous: returns after
 * enqueueing.  max_m/max_n must bound every pair's lengths (pairs that exceed them are skipped
 * with SA_FLAG_BAD_SHAPE).  d_match_lut as in sa_align_batch (device copy) or NULL.
 * d_ops must hold seq1_off[npairs] + seq2_off[npairs] + npairs bytes.
 * No LocalGotoh size hack here: this is the raw kernel path. */
int sa_align_batch_device(sa_ctx* ctx, int algo, const sa_scoring* scoring,
                          const uint8_t* d_seq1, const uint64_t* d_seq1_off,
                          const uint8_t* d_seq2, const uint64_t* d_seq2_off, uint32_t npairs,
                          uint32_t max_m, uint32_t max_n, const uint8_t* d_match_lut,
                          sa_result* d_results, uint8_t* d_ops, void* stream);

/* Device time of the kernels of the last sa_align_batch[_device] call, from HIP events
 * recorded on the stream they ran on: total fill-kernel ms, total traceback-kernel ms, and the
 * number of fill launches.  Waits for those events. */
int sa_last_timings(sa_ctx* ctx, float* fill_ms, float* traceback_ms, int* fill_launches);
// With $SEQALIB_KERNEL_TIMING set during the last call: the fill kernels alone (HIP events around
// each fill launch on its stream) and the whole fill-stream span (fill + end-cell replay, = the
// fill_ms of sa_last_timings).  SA_ERR_ARG when the last call ran without the variable.
int sa_last_kernel_timings(sa_ctx* ctx, float* fill_kernel_ms, float* fill_stream_ms);

/* Fill kernel of the last sa_align_batch[_device] call: SA_KERNEL_INT32 (int32 scores, equality
 * flags; any alphabet, LUT, scoring) or SA_KERNEL_T16 (tagged 16-bit profile kernels: SW/NW and,
 * with the affine cell, LocalGotoh/GlobalGotoh, all with allow-mismatch, <= 4 distinct symbols in
 * the batch, score range checked).  Also R and W.  Environment: SEQALIB_T16=0 forces the int32
 * kernel. */
#define SA_KERNEL_INT32 0
#define SA_KERNEL_T16 1
#define SA_KERNEL_T16_ENDCELL 2   /* T16 SW / LocalGotoh with per-chunk maxima + end-cell replay */
/* Host-buffer calls of at most 64 pairs with m <= 256, n <= 1024, m * n <= 32768 (SW / NW /
 * LocalGotoh / GlobalGotoh): one kernel fills and walks each pair in one wave (int32 cells, flags
 * in LDS), reading and writing pinned host memory.  Such a call reports 0 fill launches to
 * sa_last_timings.  Environment: SEQALIB_TINY=0 sends them through the batch kernels. */
#define SA_KERNEL_TINY 3
int sa_last_plan(sa_ctx* ctx, int* kernel, int* rows_per_lane, int* waves);
/* sa_last_plan plus what the fill stored for the traceback: SA_RECORDS_FLAGS (int32 equality
 * flags), SA_RECORDS_TAGS (T16 move tags per cell) or SA_RECORDS_SCORE_ONLY (score-only T16 SW fill:
 * per-chunk snapshots + each lane's last row per step; the traceback recomputes the blocks along
 * its path).  Environment: SEQALIB_SO=0 keeps the tagged records. */
#define SA_RECORDS_FLAGS 0
#define SA_RECORDS_TAGS 1
#define SA_RECORDS_SCORE_ONLY 2
int sa_last_plan_ex(sa_ctx* ctx, int* kernel, int* rows_per_lane, int* waves, int* records);

/* Plan of the int32 kernel for a batch (host-only query, no device needed): rows per lane R,
 * waves per workgroup W, direction bytes per pair, row-buffer bytes per pair.  The plan the
 * engine actually selects (T16 for DNA) is sa_plan_query_ex's. */
int sa_plan_query(int algo, uint32_t max_m, uint32_t max_n, uint32_t npairs,
                  int* rows_per_lane, int* waves, uint64_t* dir_bytes_per_pair,
                  uint64_t* rowbuf_bytes_per_pair);

/* Plan of a batch for a given scoring (host-only query, no device needed): the kernel the
 * engine selects when the batch holds `nsym` distinct symbols (SA_KERNEL_*; T16 needs nsym <= 4
 * and a scoring whose scores provably fit 16 bits), its R and W (W = 0: the multi-workgroup
 * plan), and the device workspace one pair occupies (direction records + row buffers + end-cell
 * snapshots; the larger of the T16 and int32 variants when the scoring admits T16, since the
 * variant is chosen on the device and both are provisioned).  A pipelined context
 * (sa_set_pipeline) holds SA_PIPELINE_DEPTH such slots per pair of a launch. */
int sa_plan_query_ex(int algo, const sa_scoring* scoring, uint32_t max_m, uint32_t max_n,
                     uint32_t npairs, int nsym, int* kernel, int* rows_per_lane, int* waves,
                     uint64_t* workspace_bytes_per_pair);

/* Tests only (tests/test_gpu_robust.py).  SA_HOOK_HAND_TAG: the band-unit hand-off tag of the
 * context's last launch becomes `value` (0..65535; the next launch takes value + 1, and at 65535 the
 * hand-off buffer is zeroed and the tags restart at 1).  SA_HOOK_POISON_WS: every 32-bit word of the
 * context's cached workspace becomes `value` (after its pending work; synchronous), as stale words
 * of earlier calls of other shapes would be.  SA_HOOK_F16: 0 / 1 allows / turns off the f16 cell of
 * the two-pairs-per-wave SW fill for the context (after its pending work); 2 returns 1 when it is
 * off (the context turned it off after a launch flagged more than 1/64 of its pairs), else 0.
 * Returns SA_OK or SA_ERR_ARG (SA_HOOK_F16 with 2: 1 / 0). */
#define SA_HOOK_HAND_TAG 1
#define SA_HOOK_POISON_WS 2
#define SA_HOOK_F16 3
int sa_test_hook(sa_ctx* ctx, int hook, uint64_t value);

/* Synthetic DNA: std::mt19937_64(seed), symbol = "ACGT"[g() & 3]. */
int sa_synth_dna(uint64_t seed, uint32_t len, uint8_t* out);
/* "Related" copy of src: per position r = g() % 100: r < 10 substitute "ACGT"[g()&3];
 * r < 12 insert "ACGT"[g()&3] before it; r < 14 delete it; else copy.  g = mt19937_64(seed).
 * Writes at most cap bytes; *out_len = produced length (may exceed cap -> SA_ERR_CAPACITY). */
int sa_synth_mutate(const uint8_t* src, uint32_t len, uint64_t seed, uint8_t* out, uint32_t cap,
                    uint32_t* out_len);
/* npairs independent pairs: pair p uses seeds base+2p+1 (seq1, len1) and base+2p+2 (seq2, len2);
 * writes concatenated sequences and npairs+1 offsets.  Uses up to `threads` host threads. */
int sa_synth_dna_batch(uint64_t base, uint32_t npairs, uint32_t len1, uint32_t len2,
                       uint8_t* seq1, uint64_t* seq1_off, uint8_t* seq2, uint64_t* seq2_off,
                       int threads);

#ifdef __cplusplus
}
#endif
#endif /* SEQALIB_HIP_H */
