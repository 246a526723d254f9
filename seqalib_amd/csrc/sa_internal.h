// sa_internal.h — parameter blocks and launcher entry points shared by the HIP translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/seqalib_hip.h"
#include "sa_layout.h"

namespace sa {

struct FillParams {
    const uint8_t* seq1;
    const uint64_t* off1;
    const uint8_t* seq2;
    const uint64_t* off2;
    const uint32_t* lutbits;   // 256 x 8 words: bit b of word [a*8 + b/32] = match(a, b)
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
    int stage_seq2;            // 1: Seq2 of the pair is copied to LDS (max_n <= kMaxStagedSeq2)
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
};

// R in {4, 8, 16}; keyed: 16-bit (score, column) max keys (local modes only).
// Returns hipSuccess or the launch error.
hipError_t launch_fill(int algo, int R, bool lut, bool allow, bool keyed, const FillParams& p,
                       uint32_t grid, hipStream_t stream);
hipError_t launch_fill_sw(int R, bool lut, bool allow, bool keyed, const FillParams& p, uint32_t grid, hipStream_t s);
hipError_t launch_fill_nw(int R, bool lut, bool allow, bool keyed, const FillParams& p, uint32_t grid, hipStream_t s);
hipError_t launch_fill_lg(int R, bool lut, bool allow, bool keyed, const FillParams& p, uint32_t grid, hipStream_t s);
hipError_t launch_fill_gg(int R, bool lut, bool allow, bool keyed, const FillParams& p, uint32_t grid, hipStream_t s);
hipError_t launch_traceback(int algo, int R, bool lut, const TbParams& p, hipStream_t stream);

}  // namespace sa
