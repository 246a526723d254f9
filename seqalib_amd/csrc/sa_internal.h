// sa_internal.h — parameter blocks and launcher entry points shared by the HIP translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/seqalib_hip.h"
#include "sa_layout.h"

namespace sa {

// How the fill decides match(Seq1[i-1], Seq2[j-1]) (sa_fill_impl.h).
constexpr int kMatchEq = 0, kMatchLut = 1, kMatchBits = 2;

// Internal per-pair flags (never returned: the int32 redo clears them).  kFlagRetry: a T16 SW
// fill found a maximum above FillParams::retry_above, where a 16-bit candidate may have wrapped,
// so the pair is re-run by the int32 variant; kFlagRedo: the int32 variant re-ran it (the T16
// end-cell replay and traceback skip it, the int32 traceback walks it).
constexpr uint32_t kFlagRetry = 1u << 30, kFlagRedo = 1u << 31;
// kFlagRerun: a SPLIT pair whose band wait expired (SA_FLAG_TIMEOUT) was re-run by the
// single-workgroup fallback plan of the same call (run_device, sa_api.hip); its traceback walks it.
constexpr uint32_t kFlagRerun = 1u << 29;
// Bounded wait of a SPLIT band for its producer, in s_memrealtime ticks (100 MHz): 0.2 s.
constexpr uint64_t kSplitWaitTicksDefault = 20000000ull;
// Polls of a band unit's hand-off word before it gives up on the producer (FillParams::wait_polls):
// a poll is one agent-scope load plus s_sleep 2, so about a second -- its producer holds a smaller
// ticket and is always running, so only a lost wave gets there.  $SEQALIB_SO_WAIT_POLLS (tests).
constexpr uint32_t kSoWaitPollsDefault = 1u << 20;

struct FillParams {
    const uint8_t* seq1;
    const uint64_t* off1;
    const uint8_t* seq2;
    const uint64_t* off2;
    const uint32_t* lutbits;   // 256 x 8 words: bit b of word [a*8 + b/32] = match(a, b)
    // kMatchBits: pair p's m x n match bitmap at mbits + mbits_off[p], row-major, ceil(n/32)
    // words per row, bit j of row i = match(Seq1[i], Seq2[j])
    const uint32_t* mbits;
    const uint64_t* mbits_off;
    uint8_t* dirs;             // direction slots, one per pair of this launch
    uint64_t dir_slot;         // bytes per slot
    uint64_t band_stride;      // bytes per band inside a slot
    int32_t* rowbuf;           // per-slot row buffer: [H or M: max_n][Ix: max_n]
    uint64_t rowbuf_slot;      // int32 elements per slot
    sa_result* res;
    uint32_t pair_base;        // first pair index of this launch
    uint32_t max_m, max_n;
    int32_t gap, match, mismatch, gap_open, gap_extend;
    int waves;                 // waves per workgroup (blockDim.x / 64)
    uint32_t count;            // pairs of this launch (the two-pair kernel's odd tail)
    int stage_seq2;            // 1: Seq2 of the pair is copied to LDS (max_n <= kMaxStagedSeq2)
    // T16 kernel only: the batch alphabet is <= 4 symbols, prof[4] = sym_pack (byte c = the
    // symbol of code c) and prof[c] holds, in byte c', the tagged substitution term
    // 4*s(sym c, sym c') + 3 as int8, 8*s + 6 for the affine kernel (written on the device by
    // decide_t16, sa_alphabet.hip).
    const uint32_t* prof;
    // device-side kernel selection: the launch runs only if *sel == sel_want (sel NULL: always);
    // redo: an int32 launch the batch did not select still re-runs the pairs flagged kFlagRetry
    const uint32_t* sel;
    uint32_t sel_want;
    int redo;
    // T16 only: NW keeps 4 * (H - t16_delta) (a constant offset that centres the score range in
    // int16); SW flags pairs whose maximum exceeds retry_above (INT_MAX when proven to fit);
    // T16 GlobalGotoh: the per-pair composition cap of a screened window (fill_kernel)
    int32_t t16_delta;
    int32_t retry_above;
    // T16 affine only: the Ix / Iy border value (the reference's -10000), encoded below every
    // candidate of the batch's score range (t16_mode, sa_api.hip)
    int32_t t16_sent;
    // CMAX only (see sa_fill_impl.h): per-slot snapshots [band][chunk][word][lane] of the R 16-bit row
    // values (R/2 words) and of the diagonal input (1 word); snap_nch = chunks per band.
    uint32_t* snap_h;   // LocalGotoh: R values of M, then R of Iy, then the last row's Ix (R + 1 words)
    int32_t* snap_p;
    int32_t* snap_m;   // per [band][chunk][lane]: the lane's maximum over the chunk (4H)
    uint64_t snap_h_slot, snap_p_slot;   // snap_m slots are snap_p_slot words too
    uint32_t snap_nch;
    // SPLIT only: one single-wave workgroup per (pair slot, band), split_bands bands per slot,
    // bands handed out by *ticket.  hand: per slot and band, max_n 8-byte {tag, H} granules of
    // the band's last row (Ix: at + hand_x_off); part: per slot and band {score, i, j, timeout}.
    unsigned long long* hand;
    uint64_t hand_x_off;
    uint32_t* ticket;
    int32_t* part;
    uint32_t split_bands;
    uint64_t wait_ticks;       // SPLIT: bounded wait for the producer band (s_memrealtime ticks)
    // the fallback launch: re-runs only the pairs a SPLIT fill flagged SA_FLAG_TIMEOUT
    int rerun;
    // score-only fills (band units, sa_fill_impl.h BU): ticket = the unit counter (zeroed before
    // the launch), epoch = this launch's tag in [1, 65535] (sa_ctx::hand_tag) of the row-buffer
    // granules, the segment state and the per-unit maxima band_part (part_bands 64-bit words per
    // slot: epoch << 48 | lost << 31 | the unit's maximum).  All three live in the context's hand-off
    // buffer, which only these fills write and which is zeroed when allocated and whenever the tag
    // wraps, so any word there carries the tag of the launch that wrote it, or none (0).
    uint32_t epoch;
    unsigned long long* band_part;
    uint32_t part_bands;
    // column segments of the band units (score-only SW / NW): every (pair, band) is cut into
    // part_segs units of consecutive chunks; a unit hands its lanes' state at its last column to
    // the next segment's unit through seg_hand (per slot: bands x segs x (R + 1) x 64 epoch-tagged
    // 16-bit values, seg_slot words).  part_segs = 1: one unit per band.
    uint32_t part_segs;
    uint32_t* seg_hand;
    uint64_t seg_slot;
    // score-only SW: per slot and (band, chunk) the wave's maximum of the chunk maxima (snap_m), so
    // the end-cell replay reads the lane maxima of the chunks that reach its threshold only
    int32_t* snap_c;
    // band units: polls of a hand-off word (row granules, segment state, per-unit maxima) before the
    // unit gives up on its producer and flags the pair for the int32 re-run (kFlagRetry)
    uint32_t wait_polls;
    // the two-pairs-per-wave SW fill (sa_fill_so2.hip): bytes of LDS per pair for its unit's Seq2
    // symbol codes (0: read from global memory per chunk)
    uint32_t so2_stage;
    // 1: its f16 cell (SW; every value exact below 2048, pairs above kSo2F16RetryAbove re-run)
    uint32_t so2_f16;
};
// the f16 cell's retry threshold on (sampled maximum - kSoSlack Gap): below it every value of the
// pair stayed below 2048 (sa_fill_so2.hip)
constexpr int32_t kSo2F16RetryAbove = 2000;

// SPLIT fills: per-pair fold of the per-band partials into sa_result (split_reduce_kernel).
struct SplitReduceParams {
    const uint64_t* off1;
    const uint64_t* off2;
    const int32_t* part;
    sa_result* res;
    uint32_t pair_base, count, split_bands, band_rows;
    uint32_t max_m, max_n;
    int32_t gap, gap_open, gap_extend;
    int cmax;
    const uint32_t* sel;
    uint32_t sel_want;
    int redo;              // as FillParams::redo
    int32_t retry_above;   // T16 SW: flag pairs with a larger maximum (kFlagRetry)
};
hipError_t launch_split_reduce(int algo, const SplitReduceParams& p, hipStream_t stream);

// End-cell replay (sa_endcell.hip) after a CMAX fill: res.reserved = chunk + 1 of the maximum.
struct EndcellParams {
    const uint8_t* seq1;
    const uint64_t* off1;
    const uint8_t* seq2;
    const uint64_t* off2;
    const uint32_t* prof;      // as FillParams::prof (prof[4] = sym_pack)
    const uint32_t* sel;
    uint32_t sel_want;
    const uint32_t* snap_h;
    const int32_t* snap_p;
    const int32_t* snap_m;
    uint64_t snap_h_slot, snap_p_slot;
    uint32_t snap_nch;
    const int32_t* rowbuf;
    uint64_t rowbuf_slot;
    uint32_t rowbuf_stride;    // int32 per column: 1 (row buffer) or 2 (SPLIT {value, tag} granules)
    uint64_t rowbuf_x_off;     // LocalGotoh: int32 offset of the Ix rows from the M rows
    uint32_t max_n;
    sa_result* res;
    uint32_t pair_base, count;
    int32_t gap, gap_open, gap_extend;
    int hshift;                // SW: snapshots / chunk maxima / top rows hold H << hshift (2 tagged, 0 SO)
    const int32_t* snap_c;     // score-only SW: per (band, chunk) maxima (FillParams::snap_c, snap_nch per band)
    uint64_t snap_c_slot;
    const uint8_t* dirs;       // score-only: the fill's edge stream (TbParams::dirs, band_stride)
    uint64_t dir_slot, band_stride;
    // the f16 SW fill's flagged-pair count of this launch (FillParams::ticket + 1; null: none) and
    // where the dense kernel's first lane posts {f16_seq, count} for the host (sa_api.hip f16 policy)
    const uint32_t* f16_count;
    unsigned long long* f16_host;
    uint32_t f16_seq;
};

struct TbParams {
    const uint8_t* seq1;
    const uint64_t* off1;
    const uint8_t* seq2;
    const uint64_t* off2;
    const uint32_t* lutbits;
    const uint8_t* dirs;
    uint64_t dir_slot;
    uint8_t* ops;
    sa_result* res;
    uint32_t pair_base, count;
    uint32_t max_m, max_n;
    int32_t gap, match, mismatch, gap_open, gap_extend;
    int allow;
    int tagged;                // record layout: 0 flags, 1 T16 max tags (sa_layout.h)
    int vrec;                  // kMatchBits fills: under fD the second flag bit is the match bit
    const uint32_t* sel;
    uint32_t sel_want;
    // Segmented traceback of SPLIT fills (sa_traceback_seg.hip); seg_mode 0 off, 1 long walks,
    // 2 every pair (tests).  hand / hand_x_off / split_bands: the fill's hand-off granules
    // (FillParams), hand_shift: 0 int32 values, 2 / 3 T16 4H / 8V; seg_rec: per slot and band
    // NST * (max_n + 1) + 1 exit records {i, j, nops, flags}; seg_fin: per slot {start_i,
    // start_j, nops, flags} of the band where the walk stopped.
    int seg_mode;
    const unsigned long long* hand;
    uint64_t hand_x_off;
    uint32_t split_bands;
    int hand_shift;
    int4* seg_rec;
    int4* seg_fin;
    int rerun;                 // the fallback launch: walks only the pairs flagged kFlagRerun
    // score-only fills (sa_traceback_so.hip): the edge stream lives in dirs (band_stride bytes per
    // band), the end-cell snapshots as FillParams, prof = the tagged T16 profile (prof[4] symbols)
    uint64_t band_stride;
    const uint32_t* snap_h;
    const int32_t* snap_p;
    uint64_t snap_h_slot, snap_p_slot;
    uint32_t snap_nch;
    const uint32_t* prof;
    int32_t t16_delta;         // score-only NW: the fill's values are H - t16_delta (the borders)
    int32_t t16_sent;          // score-only Gotoh: the tagged Ix / Iy border (FillParams::t16_sent)
    int so_lp;                 // score-only SW / NW: lanes per pair (0: kSo4DefaultLp)
    // The int32 re-run of a T16 batch walked before the T16 variant (pipelined calls walk it on the
    // fill stream, sa_api.hip tb_on_fill): keep_redo (the int32 walk) leaves kFlagRedo on the pairs
    // it walked, clear_redo (the T16 walk) skips those pairs and clears the bit (tb_release).
    int keep_redo, clear_redo;
};
// SA_FLAG_TIMEOUT: a SPLIT band's bounded wait for its producer expired (results invalid)


// R in {4, 8, 16}; keyed: 16-bit (score, column) max keys (local modes only); t16: the tagged
// 16-bit profile kernel (SW/NW with allow-mismatch, see sa_fill_impl.h).
// Returns hipSuccess or the launch error.
struct FillVariant {
    int R;
    bool lut, allow, keyed, t16, cmax, split;
    bool bits = false;   // kMatchBits (then lut is ignored)
    bool so = false;     // score-only T16 SW chunk-max fill (edge stream instead of records)
    bool so2 = false;    // score-only SW with two pairs per wave (sa_fill_so2.hip)
};
hipError_t launch_fill(int algo, const FillVariant& v, const FillParams& p, uint32_t grid, hipStream_t stream);
hipError_t launch_fill_sw(const FillVariant& v, const FillParams& p, uint32_t grid, hipStream_t s);
hipError_t launch_fill_nw(const FillVariant& v, const FillParams& p, uint32_t grid, hipStream_t s);
hipError_t launch_fill_lg(const FillVariant& v, const FillParams& p, uint32_t grid, hipStream_t s);
hipError_t launch_fill_gg(const FillVariant& v, const FillParams& p, uint32_t grid, hipStream_t s);
// Score-only SW band units with two pairs per wave (sa_fill_so2.hip), R in {16, 32}: grid =
// ceil(count / 2) x bands x part_segs units.
hipError_t launch_fill_so2(int algo, int R, const FillParams& p, uint32_t grid, hipStream_t s);
// Batch alphabet scan (presence bitmap of every byte of both sequence sets, 8 words) and the
// device-side T16 decision.  aux layout (kAux* below): [bitmap 8][profile 4][sym_pack][sel].
constexpr int kAuxProf = 8, kAuxSel = 13, kAuxWords = 64;
constexpr int kAuxTicket = 32;   // the score-only fill's unit ticket (zeroed before each launch)
constexpr int kAuxF16Flags = 33;   // the f16 SW fill's flagged pairs (zeroed with the ticket)
// Score-only SW fill: steady chunks track the lane maximum at rows and steps 3 mod 4 only, so a
// cell is at most its tracked cell - kSoSlack * gap (3 rows + 3 columns of gap moves)
constexpr int kSoSlack = 6;
// Score-only SW / NW band units: column segments per band (FillParams::part_segs).  A band of a
// 4096-column pair is ~3 ms of one wave; cut into 2 units the launch tail (the last generation of
// units draining) is half of that.  Pipelined headline step (profiles/fill_segs_ab_r05.txt):
// 1 segment 17.95 / 18.07 ms, 2: 17.51 / 17.53, 3: 17.66 / 17.64, 4: 17.75 / 17.75.
constexpr uint32_t kSoSegs = 2;
// Two pairs per wave (sa_fill_so2.hip): a unit carries two pairs' work, so the tail is twice as
// long at the same count; pipelined 10,000-pair steps by segments (profiles/so2_segs_r06.jsonl):
// 4096^2 2: 16.85-16.88 ms, 3: 16.56-16.59, 4: 16.46-16.55, 5: 16.51-16.55, 6: 16.55-16.57,
// 8: 16.45-16.49, 12: 16.58-16.62; 2048^2 2: 5.00-5.09, 4: 4.88-4.89, 8: 4.80; 1024^2 (33 chunks)
// 2: 1.66-1.70, 6: 1.63, 8: 1.64-1.65; NW 1024^2 (profiles/so2_r16_r06.jsonl) 4: 1.58, 8: 1.63-1.69,
// one pair per wave at 2: 1.61 -- so at most 8, and at least 8 chunks per segment (sa_api.hip).
// The one-pair-per-wave NW units keep 2
// (profiles/nw_segs_r06.jsonl: 1024^2 2: 1.68 ms, 4: 1.68-1.71, 8: 1.81; 4096^2 2: 17.1-17.3,
// 4: 17.2-17.3, 8: 17.9).
constexpr uint32_t kSo2Segs = 8;
hipError_t launch_alphabet_scan(const uint8_t* d1, const uint64_t* o1, const uint8_t* d2,
                                const uint64_t* o2, uint32_t npairs, uint32_t* aux, hipStream_t s);
// decide_t16: from the bitmap, aux[kAuxSel] = 1 if the batch has <= 4 distinct symbols (then the
// profile and sym_pack are written), else 0.
hipError_t launch_decide_t16(const uint32_t* lutbits, int match, int mismatch, int affine, uint32_t* aux,
                             hipStream_t s);

// Device-side kernel selection: a launch whose variant the batch did not select returns at once
// (uniform over the grid; sel NULL = unconditional).
__device__ __forceinline__ bool sa_skip(const uint32_t* sel, uint32_t want) {
    return sel != nullptr && *sel != want;
}
// Traceback of a pair: by the launch of the variant the batch selected, except the pairs the
// int32 variant re-ran (kFlagRedo), which its own traceback walks.
// A pair whose SPLIT band wait expired is walked by the fallback launch that re-ran it.
template <typename TP>
__device__ __forceinline__ bool tb_mine(const TP& P, uint32_t flags) {
    if (P.rerun) return (flags & kFlagRerun) != 0;
    if (flags & SA_FLAG_TIMEOUT) return false;
    if (!P.sel) return true;
    const bool redone = (flags & kFlagRedo) != 0;
    return *P.sel == P.sel_want ? !redone : redone;
}
// The internal flags a walk clears on a pair it walked (the results it returns carry none): all of
// them, except kFlagRedo when the T16 walk still follows (TbParams::keep_redo).
template <typename TP>
__device__ __forceinline__ uint32_t tb_clear_mask(const TP& P) {
    return ~(kFlagRetry | kFlagRerun | (P.keep_redo ? 0u : kFlagRedo));
}
// A pair tb_mine() refused: when the int32 walk ran first (TbParams::clear_redo) and re-ran this
// pair, the T16 walk leaves it to that walk's result and clears the kFlagRedo it left.  So the
// pair is walked exactly once, by the variant that filled it, whichever walk is enqueued first.
template <typename TP>
__device__ __forceinline__ void tb_release(const TP& P, sa_result* r, uint32_t flags) {
    if (P.clear_redo && (flags & kFlagRedo) && P.sel && *P.sel == P.sel_want) r->flags = flags & ~kFlagRedo;
}
// Does a pair take the segmented traceback?  The seg kernels and the wave walker evaluate it on
// the same (unchanged) sa_result, so they agree.  *b_e: the band of the walk's first cell.  Long
// walks only: a local path of score S has >= S / match diagonal moves, a global one >= max(m, n).
constexpr int kSegMinMoves = 64;
template <int ALG, int R>
__device__ __forceinline__ bool seg_take(const TbParams& P, const sa_result& res, int m, int n, int* b_e) {
    if (!P.seg_mode || !P.hand) return false;
    if (res.flags & (SA_FLAG_BAD_SHAPE | SA_FLAG_TIMEOUT)) return false;
    if (!tb_mine(P, res.flags)) return false;
    if (m <= 0 || n <= 0) return false;
    constexpr bool SCORED = (ALG == SA_SW || ALG == SA_LOCAL_GOTOH);
    int ie = m;
    if (SCORED) {
        ie = res.end_i;
        if (ie < 1 || ie > m || res.end_j < 1 || res.end_j > n) return false;
    }
    *b_e = (ie - 1) / (kWave * R);
    if (P.seg_mode == 2) return true;
    if (*b_e < 1) return false;
    if (SCORED) return P.match > 0 && (int64_t)res.score >= (int64_t)kSegMinMoves * P.match;
    return m + n >= 16 * kSegMinMoves;
}
// inject (tests only): overwrite the exit records between the two kernels
hipError_t launch_traceback_seg(int algo, int R, bool lut, const TbParams& p, hipStream_t stream, bool inject = false);
hipError_t launch_traceback(int algo, int R, bool lut, const TbParams& p, hipStream_t stream);
// One wave per pair (sa_traceback_wave.hip): the few-pairs traceback.
hipError_t launch_traceback_wave(int algo, int R, bool lut, const TbParams& p, hipStream_t stream);
hipError_t launch_endcell(int algo, int R, const EndcellParams& p, hipStream_t stream);
// Score-only SW / NW fills: the block-recompute traceback (sa_traceback_so.hip), R in {4, 8, 16, 32}.
hipError_t launch_traceback_so(int algo, int R, const TbParams& p, hipStream_t stream);
// Score-only SW fills: the end cell from the per-(band, chunk) maxima of the tracked cells.
hipError_t launch_endcell_so(int R, const EndcellParams& p, hipStream_t stream);

// The small-call path (sa_tiny.hip): one single-wave workgroup per pair fills, keeps the flags
// in LDS and walks the traceback; inputs and outputs are pinned host memory mapped into the GPU.
// Shapes: m <= kTinyM, n <= kTinyN, m * n <= kTinyCells, at most kTinyPairs pairs per call.
constexpr int kTinyM = 256, kTinyN = 1024, kTinyCells = 32768, kTinyPairs = 64;
struct TinyParams {
    const uint8_t* seq1;
    const uint64_t* off1;      // npairs + 1 offsets (prefix sums)
    const uint8_t* seq2;
    const uint64_t* off2;
    const uint32_t* lutbits;   // 2048 words, or NULL (identity)
    sa_result* res;
    uint8_t* ops;              // pair p's ops at off1[p] + off2[p] + p
    uint32_t npairs;
    int32_t gap, match, mismatch, gap_open, gap_extend;
    int allow;
};
hipError_t launch_tiny(int algo, bool lut, int max_m, const TinyParams& p, hipStream_t stream);
}  // namespace sa
