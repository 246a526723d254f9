/* TEST INFRASTRUCTURE ONLY — the CPU checker for the product's HIP path.
 *
 * Clean-room C restatement of the reference's four DP aligners (przemektmalon/SeqALib):
 *   SmithWatermanSA  (include/SASmithWaterman.h:20-366)
 *   NeedlemanWunschSA(include/SANeedlemanWunsch.h:22-264)
 *   LocalGotohSA     (include/SALocalGotoh.h:36-526, incl. the size hack :484-488)
 *   GlobalGotohSA    (include/SAGlobalGotoh.h:33-459)
 * plus SequenceAligner::forceGlobal (include/SequenceAlignment.h:156-189)
 * and HirschbergSA (include/SAHirschberg.h:11-184; score = NW H[m][n], the reference reports none)
 * and MyersMillerSA (include/SAMyersMiller.h:43-420; score = the top call's optimum, see
 * align_myers_miller; the reference reports none).
 *
 * Parity is PINNED: tests/test_oracle_golden.py checks this restatement against golden vectors
 * produced by the unmodified reference (oracle/_ref, tests/golden/make_golden.py).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / baseline — never as the product path.
 */
#ifndef SA_ORACLE_H
#define SA_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_SW = 0, OR_NW = 1, OR_LOCAL_GOTOH = 2, OR_GLOBAL_GOTOH = 3, OR_HIRSCHBERG = 4, OR_MYERS_MILLER = 5 };

typedef struct {
    int32_t gap, match, mismatch, gap_open, gap_extend, allow_mismatch;
} oracle_scoring;

typedef struct {
    int32_t score;           /* SW/LG: max score; NW/GG: H[m][n] */
    int32_t end_i, end_j;    /* SW/LG: (MaxRow, MaxCol); NW/GG: (m, n) */
    int32_t start_i, start_j;/* (i, j) where the traceback stopped */
    int32_t nops;            /* number of traceback ops written (traceback order) */
    int32_t len;             /* number of AlignedSequence entries after forceGlobal */
} oracle_result;

/* Op codes of the traceback stream, in the order the reference's buildResult emits them
 * (push_front order, i.e. from the end cell backwards):
 *   'M' diag, match fn true        'S' diag, match fn false
 *   'U' up   (Seq1[i-1], Blank)    'L' left (Blank, Seq2[j-1])
 *   'X' diag with !AllowMismatch and no match: emits (Seq1[i-1],Blank) then (Blank,Seq2[j-1])
 *   'u' / 'l' LocalGotoh gap-open emitted without moving, then break (SALocalGotoh.h:395-400, :451-456)
 */

/* Align one pair.  lut: 256x256 match table indexed [s1 byte][s2 byte] (NULL = byte equality).
 * Writes up to ops_cap ops and, if row0 != NULL, up to cap entries as three strings
 * (Entry.get(0), '|'/' ' for Entry.match(), Entry.get(1); Blank is '-').
 * Returns 0 on success, -1 if a buffer was too small, -2 on allocation failure. */
int oracle_align(int algo, const oracle_scoring* sc, const uint8_t* s1, int m, const uint8_t* s2,
                 int n, const uint8_t* lut, oracle_result* res, uint8_t* ops, int ops_cap,
                 char* row0, char* bars, char* row1, int cap);

/* CPU baseline ("port"): SW over a batch of pairs on `threads` threads, full reference-shaped
 * computation (bool match cache, int32 row-major matrix, traceback, forceGlobal).
 * Writes each pair's max score into out_score.  Returns 0 or -2. */
int oracle_batch(int algo, const oracle_scoring* sc, const uint8_t* s1cat, const uint64_t* off1,
                 const uint8_t* s2cat, const uint64_t* off2, int npairs, int threads,
                 oracle_result* res, uint8_t* ops);
int oracle_sw_score_batch(const oracle_scoring* sc, const uint8_t* s1cat, const uint64_t* off1,
                          const uint8_t* s2cat, const uint64_t* off2, int npairs, int threads,
                          int32_t* out);
int oracle_align_matrix(int algo, const oracle_scoring* sc, int m, int n, const uint8_t* mt,
                        oracle_result* res, uint8_t* ops, int ops_cap);
int oracle_sw_batch(const oracle_scoring* sc, const uint8_t* s1cat, const uint64_t* off1,
                    const uint8_t* s2cat, const uint64_t* off2, int npairs, int threads,
                    int32_t* out_score);

#ifdef __cplusplus
}
#endif
#endif
