// recon_kernel.h — device side of the macroblock reconstruct path (gfx950 / CDNA4).
//
// One workgroup (4 waves) per slice = MB row (XCD-aware slice order); each wave reconstructs
// groups of 4 consecutive macroblocks (groups w, w+4, w+8, ... of the row) with wave-private LDS,
// so no workgroup barrier sits in the loop, which is software-pipelined one group ahead.  Per
// group (recon.hip has the details):
//   1. dequant + mismatch control         reference mb_decoder.cpp:74-155 (parse_block)
//      lane = coefficient word (coalesced 4-B loads, prefetched one group ahead), scattered into
//      compacted coded-block slots in LDS through a per-group dequant table.
//   2. IDCT, SSE2-exact                    reference idct_sse2.hpp:23-120
//      lane = two lines of one block on packed i16 pairs; the block parity (mismatch control)
//      is reduced over the block's 4 lanes with ds_swizzle; pass 1, transpose in LDS, pass 2,
//      >>6 -> residual image with the dct_type placement of mb_decoder.cpp:166-196.
//   3. MC + add/clip + store               reference mb_decoder.cpp:198-339, mc_sse2.hpp,
//      idct_sse2.hpp:106-119 (packus / adds+packus)
//      lane = one pixel row (16-px luma, 8/16-px chroma): reference rows by raw buffer loads
//      issued one group ahead, cascaded half-pel averages with v_lerp_u8 (== _mm_avg_epu8),
//      bidirectional average, residual add + clamp on packed i16, one 16-B / 8-B row store.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mp2vg.h"

namespace mp2vg {

struct SliceDesc {
    uint32_t pic;       // index into the batch's picture array
    uint32_t mb_begin;  // first MB record (absolute)
    uint32_t mb_count;
    uint32_t reserved;
};

// one kernel launch: a slice range of one dependency level and one motion-compensation mode
// (0: I pictures, 1: P, forward only, 2: B, 3: P and B, 4: I pictures without tile stores)
struct Launch {
    uint32_t begin, end;
    int mcm;
    int mates = 0;  // consecutive one-row slices (cluster mates) per workgroup: 0 / 2 / 4
    int level;  // dependency level: launches of one level may run concurrently
    int set;    // independent picture set (its own stream)
};

// per-launch geometry, passed by value
struct Geo {
    uint8_t* sink;  // 16+ writable, readable bytes outside every slot: dummy loads and stores
    uint64_t slot_bytes;   // one picture (frame_c layout); a slot's anchor tiles are 2 x this
    const uint64_t* ftab;  // device address of frame slot i (the frame pool's slot table)
    const uint64_t* ttab;  // device address of slot i's anchor tiles
    uint32_t plane_off[3];  // plane offsets inside a slot (a slot is < 4 GiB)
    int32_t stride[3];
    int32_t ph[3];
};

struct KArgs {
    const mp2vg_picture_t* pics;
    const mp2vg_mb_t* mbs;
    const uint32_t* coefs;
    const SliceDesc* slices;
    uint8_t* sink;
    uint64_t slot_bytes;
    const uint64_t *ftab, *ttab;
    uint64_t plane_off[3];
    int32_t stride[3];
    int32_t ph[3];
    uint32_t slice_base;
    uint32_t nslices;
    uint32_t mates = 0;  // P/B launches: consecutive slices per workgroup, 2 or 4 (Launch.mates)
};

// decoded slots -> host (or HBM) frames of one drop-in chunk, by a copy kernel (recon.hip);
// 16-B aligned pointers, kernel arguments by value
constexpr int kFrameCopyMax = 32;
struct FrameCopy {
    const uint8_t* src[kFrameCopyMax];
    uint8_t* dst[kFrameCopyMax];
};
hipError_t launch_frame_copy(const FrameCopy& fc, int n, uint64_t bytes, hipStream_t stream);

}  // namespace mp2vg
