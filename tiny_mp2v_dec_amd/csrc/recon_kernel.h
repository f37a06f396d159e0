// recon_kernel.h — device side of the macroblock reconstruct path (gfx950 / CDNA4).
//
// One workgroup (4 waves) per slice = MB row; each wave reconstructs whole macroblocks
// independently (MBs w, w+4, w+8, ... of the row) with wave-private LDS, so no workgroup barrier
// sits in the MB loop.  Per macroblock:
//   1. dequant + mismatch control         reference mb_decoder.cpp:74-155 (parse_block)
//      lanes = coefficient words (coalesced 4-B loads), LDS scatter into a per-block raster,
//      mismatch parity by LDS xor atomics.
//   2. IDCT, SSE2-exact                    reference idct_sse2.hpp:23-120
//      lane = (block, line): pass 1 over the horizontal frequency (one 16-B LDS row read),
//      LDS transpose, pass 2, >>6 -> residual image in LDS with the dct_type placement of
//      mb_decoder.cpp:166-196.
//   3. MC + add/clip + store               reference mb_decoder.cpp:198-339, mc_sse2.hpp,
//      idct_sse2.hpp:106-119 (packus / adds+packus)
//      lane = 4 horizontally adjacent pixels: 4-byte SWAR half-pel averaging with the
//      reference's cascaded rounding, bidirectional average, residual add + clamp, one
//      4-byte store.
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
// (0: I pictures, 1: P, forward only, 2: B)
struct Launch {
    uint32_t begin, end;
    int mcm;
    int level;  // dependency level: launches of one level may run concurrently
    int set;    // independent picture set (its own stream)
};

// per-launch geometry, passed by value
struct Geo {
    uint8_t* sink;  // 16+ writable, readable bytes outside every slot: dummy loads and stores
    uint64_t slot_bytes;
    uint32_t plane_off[3];  // plane offsets inside a slot (a slot is < 4 GiB)
    int32_t stride[3];
    int32_t ph[3];
};

struct KArgs {
    const mp2vg_picture_t* pics;
    const mp2vg_mb_t* mbs;
    const uint32_t* coefs;
    const SliceDesc* slices;
    uint8_t* pool;
    uint8_t* sink;
    uint64_t slot_bytes;
    uint64_t plane_off[3];
    int32_t stride[3];
    int32_t ph[3];
    uint32_t slice_base;
    uint32_t nslices;
};

}  // namespace mp2vg
