// sa_layout.h — geometry shared by the fill kernel, the traceback kernel and the host planner.
//
// One workgroup aligns one pair.  The DP matrix (rows i = Seq1, cols j = Seq2, 1-based cells) is
// cut into horizontal BANDS of 64*R rows; inside a band each of the 64 lanes of a wave owns R
// consecutive rows in registers and the wave sweeps the columns as an anti-diagonal wavefront:
// at STEP s, lane t computes column j = s - t (0-based), receiving the row-above value from lane
// t-1 through a DPP wave_shr:1.  A band therefore takes n + 63 steps.  The W waves of the
// workgroup take bands round-robin and run as a software pipeline, handing the band's last row
// to the next band through a per-pair row buffer (see sa_fill_impl.h).
//
// Instead of the reference's int32 score matrices (SASmithWaterman.h:55, SALocalGotoh.h:64-66)
// the fill writes only what the traceback needs: per cell BPC flag bits
//   linear (SW/NW), BPC = 2:  fD = (H == diag term), fU = (H == up term)
//   affine (Gotoh), BPC = 4:  fD = (M == diag term), fX = (M == Ix),
//                             fXe = (Ix == Ix_up + GE), fYe = (Iy == Iy_left + GE)
// or, for the tagged 16-bit linear kernel (TAGGED records, BPC = 2), the 2-bit tag that won the
// cell's max: 3 = diag, 2 = up, 1 = left, 0 = zero clamp (sa_fill_impl.h, "T16"); for the tagged
// affine kernel (BPC = 8, one byte per cell): bit 0 = Ix extends, bit 1 = Iy extends, bits 3-4 =
// the class that won M's max: 3 = diag, 2 = Ix, 1 = Iy, 0 = zero clamp (bits 2, 5-7: don't care).
// The traceback re-derives the cell scores along its path from the end score (every move is an
// exact equality), so zero tests and gap-open clamps need no stored bits.
//
// Per band, per step, per lane a record of R*BPC bits is built by shifting flags in (flags: first
// flag of row 0 ends up most significant; tags: row r lands at bits 2r); records are grouped into
// 16-byte packets so every store is one coalesced 1 KiB wave instruction:
//   packet(b, s, half) = b*band_stride + ((s / SPP) * PPS + half) * 1024, lane t at +16*t,
//   step s at +(s % SPP)*BPS inside the lane's 16 bytes.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SA_HD __host__ __device__ __forceinline__
#else
#define SA_HD inline
#endif

namespace sa {

constexpr int kWave = 64;   // CDNA wavefront
constexpr int kChunk = 32;  // steps between workgroup barriers
// Phases a band lags its producer band: its chunk k reads columns [kC, kC+C) of the hand-off,
// which the producer wrote at the END of its chunk floor((c+63)/C) (lane 63 reaches column c at
// step c+63) -> floor((C+62)/C) chunks later, +1 for the barrier.
constexpr int kLagPhases = (kChunk + 62) / kChunk + 1;
// LDS hand-off ring (columns).  Within one phase the producer writes columns [kC-63, kC-31) while
// its consumer reads [kC-96, kC-64): disjoint and 64 apart; a slot is rewritten (column c+kRing)
// at producer chunk floor((c+kRing+63)/C) >= floor(c/C) + 5 > the consumer's read phase
// floor(c/C) + kLagPhases, so 128 columns never alias a pending read.
constexpr int kRing = 128;
static_assert(kLagPhases == 3 && kRing >= 4 * kChunk, "re-derive the ring bound");

// Per-wave step buffers of the fill (sa_fill_impl.h, "LDS-fed steps"), int32 words:
//   [0, 32) lane-0 row-above input of the chunk's steps, [32, 64) its Ix (affine),
//   [64, 96) the column symbols, [96, 128) the band's last row parked per step (H),
//   [128, 160) the same for Ix, [160, 224) the discard target of lanes 0..62's parking writes.
constexpr int kStepBufWords = 224;
// Dynamic LDS of the fill kernel: [match bits (LUT)][hand-off rings][step buffers][staged Seq2].
struct LdsLayout {
    uint32_t ring_off, step_off, seq_off, total;
};
SA_HD LdsLayout lds_layout(bool lut, bool affine, int W, uint32_t staged_n) {
    LdsLayout L;
    L.ring_off = lut ? 2048 * 4 : 0;
    L.step_off = L.ring_off + (uint32_t)W * (affine ? 2 : 1) * kRing * 4;
    L.seq_off = L.step_off + (uint32_t)W * kStepBufWords * 4;
    L.total = L.seq_off + ((staged_n + 15) / 16) * 16;
    return L;
}
// LDS a workgroup may allocate on gfx950 (MI355X_MICROARCH.md: 160 KiB per CU, all of it to one
// workgroup).
constexpr uint32_t kMaxLds = 160 * 1024;
// Seq2 is staged in LDS when it fits this budget (else read from global per chunk).
constexpr uint32_t kMaxStagedSeq2 = 48 * 1024;

SA_HD constexpr bool is_affine(int algo) { return algo >= 2; }
SA_HD constexpr int bits_per_cell(int algo) { return is_affine(algo) ? 4 : 2; }
// Record bits per cell in HBM: the flag bits, padded (above them) to 4 bits at R = 2 and 8 bits at
// R = 1, so that one lane's record of one step is always at least a byte.  R = 1 and 2 are the
// few-pairs (SPLIT) plans: their bands are short so that a lone wave's critical-path step stays
// cheap, and their records are a negligible share of the HBM traffic.
// Tagged affine records (T16 Gotoh) are one byte per cell at every R.
SA_HD constexpr int record_bpc(int algo, int R, bool tagged = false) {
    return (tagged && is_affine(algo)) ? 8 : (R == 1 ? 8 : (R == 2 ? 4 : bits_per_cell(algo)));
}
// The equality flags of the int32 affine records (bit 3 fD, bit 2 fX, bit 1 fXe, bit 0 fYe) from a
// tagged affine record byte: the class that won M's max, taken in the reference's order (diag,
// then Ix, then Iy: SALocalGotoh.h:304-468), says the same thing as the first flag that holds.
SA_HD constexpr uint32_t t16a_flags(uint32_t b) {
    return (((b >> 3) & 3u) == 3u ? 8u : 0u) | (((b >> 3) & 3u) == 2u ? 4u : 0u) | ((b & 1u) << 1) | ((b >> 1) & 1u);
}

struct Geom {
    int R;              // rows per lane
    int bpc;            // bits per cell
    int bps;            // bytes per step record per lane = R*bpc/8
    int spp;            // step records per 16-byte packet
    int pps;            // packets per step record
    uint32_t steps_pad; // steps per band, padded (multiple of kChunk)
    uint32_t bands;     // bands for max_m
    uint64_t band_stride;  // bytes per band
    uint64_t dir_slot;     // bytes per pair
    int tagged;            // 0 equality flags; 1 max tags (T16 kernels); 2 score-only edge stream
};
constexpr int kGeomEdge = 2;   // Geom::tagged of a score-only (SO) fill: 16 bits per lane-step (affine: 32)

SA_HD uint32_t round_up(uint32_t x, uint32_t a) { return (x + a - 1) / a * a; }

SA_HD Geom make_geom(int algo, int R, uint32_t max_m, uint32_t max_n, int tagged = 0) {
    Geom g;
    g.R = R;
    g.tagged = tagged;
    g.bpc = record_bpc(algo, R, tagged != 0);
    // score-only fills (sa_fill_impl.h SO) store the lane's last row per step instead of flags
    g.bps = tagged == kGeomEdge ? (is_affine(algo) ? 4 : 2) : R * g.bpc / 8;   // (affine: M and Ix)
    g.spp = g.bps >= 16 ? 1 : 16 / g.bps;
    g.pps = g.bps > 16 ? g.bps / 16 : 1;
    g.steps_pad = round_up(max_n + 63, kChunk);
    g.bands = (max_m + kWave * R - 1) / (kWave * R);
    g.band_stride = (uint64_t)g.steps_pad * kWave * (uint64_t)g.bps;
    g.dir_slot = (uint64_t)g.bands * g.band_stride;
    return g;
}

// Bit index, inside its 32-bit record word, of the least significant bit of row r's group.
// Flags: rows are pushed r = 0..R-1, BPC flags each, into words of min(32, R*BPC) bits, first row
// most significant.  Tags: v_alignbit pushes each row in at the top, so row r ends at bits 2r.
SA_HD void cell_word_bit(int R, int bpc, int r, int* word, int* lowbit, int tagged = 0) {
    const int rb = R * bpc;
    const int wb = rb < 32 ? rb : 32;
    const int rpw = wb / bpc;
    *word = r / rpw;
    *lowbit = tagged ? bpc * (r % rpw) : wb - bpc * ((r % rpw) + 1);
}

// Byte offset (inside a pair's slot) and bit shift of the flag group of cell (i, j), 1-based.
SA_HD uint64_t cell_byte(const Geom& g, uint32_t i, uint32_t j, int* shift) {
    const uint32_t ii = i - 1;
    const uint32_t band_rows = (uint32_t)kWave * g.R;
    const uint32_t b = ii / band_rows;
    const uint32_t rem = ii - b * band_rows;
    const uint32_t t = rem / g.R;
    const int r = (int)(rem - t * g.R);
    const uint32_t s = (j - 1) + t;
    int word, lowbit;
    cell_word_bit(g.R, g.bpc, r, &word, &lowbit, g.tagged);
    const uint32_t byte_in_rec = (uint32_t)word * 4 + (uint32_t)lowbit / 8;
    *shift = lowbit % 8;
    const uint32_t half = byte_in_rec / 16;
    const uint64_t packet = (uint64_t)(s / g.spp) * g.pps + half;
    return (uint64_t)b * g.band_stride + packet * (kWave * 16) + (uint64_t)t * 16 +
           (uint64_t)(s % g.spp) * g.bps + (byte_in_rec % 16);
}

// Band schedule of the workgroup software pipeline.  Wave w owns bands w, w+W, ...; band b
// starts at phase start(b) = (b / W) * period + (b % W) * kLagPhases with
// period = max(nch, W * kLagPhases), which keeps every band >= kLagPhases behind its producer
// and never schedules two bands on one wave at once.
SA_HD uint32_t chunks_per_band(uint32_t n) { return (n + 63 + kChunk - 1) / kChunk; }
SA_HD uint32_t sched_period(uint32_t nch, int W) {
    uint32_t p = (uint32_t)W * kLagPhases;
    return nch > p ? nch : p;
}
SA_HD uint32_t band_start(uint32_t b, int W, uint32_t period) {
    return (b / W) * period + (b % W) * kLagPhases;
}
SA_HD uint32_t total_phases(uint32_t bands, uint32_t n, int W) {
    if (bands == 0) return 0;
    const uint32_t nch = chunks_per_band(n);
    return band_start(bands - 1, W, sched_period(nch, W)) + nch;
}

}  // namespace sa
