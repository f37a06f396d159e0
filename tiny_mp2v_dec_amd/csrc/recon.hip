// recon.hip — HIP kernels of the macroblock reconstruct path (gfx950 / CDNA4 only: wave64,
// packed 16-bit VALU, v_lerp_u8, LDS per wave; no CUDA-compat layer).  See recon_kernel.h for
// the map to the reference.
//
// Work decomposition: one workgroup (4 waves) per slice (= MB row, XCD-aware order), or in P/B
// launches two slices of reference-sharing pictures, two waves each (`mates`); each wave
// reconstructs groups of G = 4 consecutive macroblocks with wave-private LDS:
//   A  group records (scalar loads) + first 64 coefficient words
//   B  reference-row loads for every pixel row of the group (one lane per row: 16-px luma rows,
//      8/16-px chroma rows), issued before the transform so their latency hides behind it
//   C  dequant: lanes = coefficient words -> coded-block slots (compacted) in LDS
//   D  SSE2-exact IDCT on packed i16 pairs (two lines per lane, v_pk_add_i16 clamp =
//      _mm_adds_epi16), mismatch control folded into pass 1 (ds_swizzle parity reduce)
//   E  prediction (cascaded half-pel with v_lerp_u8 == _mm_avg_epu8, bidir average) + residual
//      with clamp (packed i16) and one 16-B / 8-B store per row
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <stdint.h>
#include <stdlib.h>

#include "recon_kernel.h"

namespace mp2vg {

typedef short short2_t __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------------------------------
// SSE2 16-bit semantics on packed pairs (two independent IDCT lines per lane):
//   _mm_adds/_mm_subs_epi16 saturate, _mm_slli_epi16 wraps, _mm_mulhi_epi16 = (a*b)>>16
__device__ __forceinline__ short2_t adds2(short2_t a, short2_t b) { return __builtin_elementwise_add_sat(a, b); }
__device__ __forceinline__ short2_t subs2(short2_t a, short2_t b) { return __builtin_elementwise_sub_sat(a, b); }
__device__ __forceinline__ short2_t shl2(short2_t a, int n) {
    return __builtin_bit_cast(short2_t, __builtin_bit_cast(ushort2, a) << (unsigned short)n);
}
// _mm_mulhi_epi16 on a packed pair: two 24-bit products (SDWA word selects, full rate) and one
// v_perm of their high halves
__device__ __forceinline__ short2_t mulhi2(short2_t a, int c) {
    const uint32_t u = __builtin_bit_cast(uint32_t, a);
    const int lo = (int)(short)(u & 0xffffu) * c, hi = ((int)u >> 16) * c;
    return __builtin_bit_cast(short2_t, __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x07060302u));
}
// _mm_slli_epi16(_mm_mulhi_epi16(a, c), 1) = high halves of a*2c with bit 0 cleared: one perm and
// one AND instead of two shifts, a perm and an AND
__device__ __forceinline__ short2_t mulhi2_x2(short2_t a, int c) {
    const short2_t h = mulhi2(a, 2 * c);
    return __builtin_bit_cast(short2_t, __builtin_bit_cast(uint32_t, h) & 0xfffefffeu);
}

// idct_sse2.hpp:23-65, two lanes of the SSE2 vector at once.
// P1: the first pass over dequantised coefficients.  Every input but QFS[0] (s[0] of the rows-0/1
// item: the intra DC or the unclamped '1s' coefficient) is clamped to [-2048, 2047] by dequant
// (mb_decoder.cpp:146; mismatch control only flips bit 0 of QFS[63]), and for |a| <= 8191
//   adds(mulhi(a, c), slli(a, n)) = floor(a * (c + 2^(16+n)) / 2^16)   (no wrap, no saturation)
//   adds(slli(mulhi(a, c), 1), slli(a, n)) = 2 * floor(a * (c + 2^(15+n)) / 2^16)
// so the first-stage terms of s[1..5] are one mulhi each (two products and a perm) instead of a
// mulhi, a packed shift and a saturating packed add.  s[0] keeps the exact form.  The bounds and
// the whole folded transform are checked against the exact one in tests/test_idct_fold.py.
template <bool P1 = false>
__device__ __forceinline__ void idct_1d(short2_t s[8]) {
    const short2_t v15 = adds2(mulhi2_x2(s[0], 27145), shl2(s[0], 1));
    const short2_t v26 = P1 ? mulhi2(s[1], -5037 + 262144) : adds2(mulhi2(s[1], -5037), shl2(s[1], 2));
    const short2_t v21 = P1 ? mulhi2(s[2], -19954 + 262144) : adds2(mulhi2(s[2], -19954), shl2(s[2], 2));
    const short2_t v28 = P1 ? mulhi2_x2(s[3], -22089 + 131072) : adds2(mulhi2_x2(s[3], -22089), shl2(s[3], 2));
    const short2_t v16 = P1 ? mulhi2_x2(s[4], 27145 + 65536) : adds2(mulhi2_x2(s[4], 27145), shl2(s[4], 1));
    const short2_t v25 = P1 ? mulhi2(s[5], 14567 + 131072) : adds2(mulhi2(s[5], 14567), shl2(s[5], 1));
    const short2_t v22 = adds2(mulhi2_x2(s[6], 17391), s[6]);
    const short2_t v27 = mulhi2_x2(s[7], 25570);
    const short2_t v19 = subs2(v25, v28);
    const short2_t v20 = subs2(v26, v27);
    const short2_t v23 = adds2(v26, v27);
    const short2_t v24 = adds2(v25, v28);
    const short2_t v7 = adds2(v23, v24);
    const short2_t v11 = adds2(v21, v22);
    const short2_t v13 = subs2(v23, v24);
    const short2_t v17 = subs2(v21, v22);
    const short2_t v8 = adds2(v15, v16);
    const short2_t v9 = subs2(v15, v16);
    const short2_t v18 = mulhi2(subs2(v19, v20), 25079);              // op4
    // op3, op0: a + mulhi(a, c) = mulhi(a, c + 2^16) in pass 1 (|v19| <= 11,363, |v13| <= 20,998,
    // |v17| <= 10,703 there: no saturation, products below 2^31)
    const short2_t v12 = subs2(v18, P1 ? mulhi2(v19, 20090 + 65536) : adds2(v19, mulhi2(v19, 20090)));  // op3
    const short2_t v14 = subs2(subs2(v20, mulhi2(v20, 30068)), v18);  // op1
    const short2_t v6 = subs2(shl2(v14, 1), v7);
    const short2_t v5 = subs2(P1 ? mulhi2(v13, 27145 + 65536) : adds2(v13, mulhi2(v13, 27145)), v6);    // op0
    const short2_t v4 = adds2(v5, shl2(v12, 1));
    const short2_t v10 = subs2(P1 ? mulhi2(v17, 27145 + 65536) : adds2(v17, mulhi2(v17, 27145)), v11);  // op0
    const short2_t v0 = adds2(v8, v11);
    const short2_t v1 = adds2(v9, v10);
    const short2_t v2 = subs2(v9, v10);
    const short2_t v3 = subs2(v8, v11);
    s[0] = adds2(v0, v7);
    s[1] = adds2(v1, v6);
    s[2] = adds2(v2, v5);
    s[3] = subs2(v3, v4);
    s[4] = adds2(v3, v4);
    s[5] = subs2(v2, v5);
    s[6] = subs2(v1, v6);
    s[7] = subs2(v0, v7);
}

// two 8 x int16 lines (16 B each) -> 8 packed pairs (a[u], b[u])
__device__ __forceinline__ void interleave(const uint4& a, const uint4& b, short2_t s[8]) {
    const uint32_t av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 4; i++) {
        s[2 * i] = __builtin_bit_cast(short2_t, __builtin_amdgcn_perm(bv[i], av[i], 0x05040100u));
        s[2 * i + 1] = __builtin_bit_cast(short2_t, __builtin_amdgcn_perm(bv[i], av[i], 0x07060302u));
    }
}

// scan position -> raster (v*8+u), zig-zag / alternate (reference scan_c.cpp:41-57)
__constant__ uint8_t c_scan_raster[2][64] = {
    {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
     41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
     30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63},
    {0,  8,  16, 24, 1,  9,  2,  10, 17, 25, 32, 40, 48, 56, 57, 49, 41, 33, 26, 18, 3,  11,
     4,  12, 19, 27, 34, 42, 50, 58, 35, 43, 51, 59, 20, 28, 5,  13, 6,  14, 21, 29, 36, 44,
     52, 60, 37, 45, 53, 61, 22, 30, 7,  15, 23, 31, 38, 46, 54, 62, 39, 47, 55, 63}};

// intra-wave LDS hand-off (HIP's __syncwarp lowering: wavefront fences around a wave barrier)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// _mm_packus_epi16 on one packed pair: gfx950's v_sat_pk_u8_i16 (VOP1, full rate) clamps both i16
// halves to [0, 255] and packs them into bytes 0-1 (no clang builtin: inline asm)
__device__ __forceinline__ uint32_t sat_pk_u8(short2_t v) {
    uint32_t r;
    asm("v_sat_pk_u8_i16 %0, %1" : "=v"(r) : "v"(__builtin_bit_cast(uint32_t, v)));
    return r;
}

// per-byte (a + b + 1) >> 1 on 4 packed u8 == _mm_avg_epu8: one v_lerp_u8 (rounding bit per byte)
__device__ __forceinline__ uint32_t avg4(uint32_t a, uint32_t b) { return __builtin_amdgcn_lerp(a, b, 0x01010101u); }

// v_mul_u32_u24 (low 32 bits of a 24 x 24-bit product, full rate) as asm: on plain products the
// compiler emits quarter-rate v_mul_lo_u32 where it cannot bound an operand (a row index times a
// runtime stride) or where it re-associates (the dequant W*qs*level chain)
__device__ __forceinline__ uint32_t mul24_asm(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <int CF>
struct Fmt {
    static constexpr int NB = CF == 1 ? 6 : (CF == 2 ? 8 : 12);  // blocks per MB
    static constexpr int CW = CF == 3 ? 16 : 8;                  // chroma MB width
    static constexpr int CH = CF == 1 ? 8 : 16;                  // chroma MB height
};

// origin of block b in its MB plane image and its row step (mb_decoder.cpp:176-195)
template <int CF>
__device__ __forceinline__ void block_origin(int b, bool dctf, int& plane, int& x0, int& y0, int& ys) {
    ys = 1;
    if (b < 4) {
        plane = 0;
        x0 = (b & 1) * 8;
        if (dctf) {
            y0 = b >> 1;
            ys = 2;
        } else {
            y0 = (b >> 1) * 8;
        }
        return;
    }
    plane = (b & 1) ? 2 : 1;
    const int k = (b - 4) >> 1;
    x0 = k >= 2 ? 8 : 0;
    const bool lower = (k & 1);
    if (dctf && CF != 1) {
        y0 = lower ? 1 : 0;
        ys = 2;
    } else {
        y0 = lower ? 8 : 0;
    }
}

// the block covering the left (x<8) half of MB-plane row py; the right half is +1 (luma) or
// +4 (4:4:4 chroma: blocks 4/8, 6/10, 5/9, 7/11)
template <int CF>
__device__ __forceinline__ int left_block(int plane, int py, bool dctf) {
    const int lower = dctf ? (py & 1) : (py >> 3);
    if (plane == 0) return lower * 2;
    const int base = plane == 1 ? 4 : 5;
    if (CF == 1) return base;
    return base + 2 * lower;
}


constexpr int WAVES = 4;
constexpr int G = 4;               // macroblocks per wave group
// waves per workgroup of the I kernels (MP2VG_I_WAVES, round-5 A/B; the P/B kernels keep WAVES):
// a 1080p row is 30 groups, 8/8/7/7 over 4 waves, 5/5/5/5/5/5 over 6
#ifndef MP2VG_I_WAVES
#define MP2VG_I_WAVES 4
#endif
// I kernels: the (MB, block) -> block address table of the intra dequant (Lds::kbtab; dev A/B)
#ifndef MP2VG_I_KBTAB
#define MP2VG_I_KBTAB 1
#endif
template <int MCM, int ABL>
constexpr int kernel_waves() { return (MCM == 0 || MCM == 4) && ABL == 0 ? MP2VG_I_WAVES : WAVES; }

// Residual image of one MB in LDS (int16): luma 16x16, then Cb CW x CH, then Cr.  Inside each
// group of 4 pixels the order is x0, x0+2, x0+1, x0+3: one v_perm unpacks the matching
// prediction bytes into (x0, x0+2) / (x0+1, x0+3) pairs for packed i16 math, and IDCT pass 2
// (columns x, x+2 per lane) stores one dword per output row.
template <int CF>
struct ResLayout {
    using F = Fmt<CF>;
    static constexpr int SIZE = 256 + 2 * F::CW * F::CH;
    // MB stride of the P/B kernels' int16 image: SIZE alone is a multiple of 256 B, so the four
    // MBs' images alias the same LDS banks (the store pass reads row py of MB k, k = 0..3, in one
    // instruction); 16 B of padding spread them over the banks.  (The I kernels' byte image keeps
    // SIZE: its capacity sets their occupancy.)
#ifndef MP2VG_RES_PAD
#define MP2VG_RES_PAD 0  // 8 measured neutral (c2 381.5k/381.7k vs 382.6k/380.7k, profiles/r6/README.md)
#endif
    static constexpr int MBS = SIZE + MP2VG_RES_PAD;
    __device__ static constexpr int base(int plane) { return plane == 0 ? 0 : 256 + (plane - 1) * F::CW * F::CH; }
    __device__ static constexpr int width(int plane) { return plane == 0 ? 16 : F::CW; }
    __device__ static int pos(int x) { return (x & ~3) | ((x & 1) << 1) | ((x >> 1) & 1); }
};

// select one of three wave-uniform per-plane values by a lane-varying plane index (plain
// indexing makes the compiler re-load the kernel-argument array with per-lane vector loads)
template <class T>
__device__ __forceinline__ T gsel(const T (&v)[3], int plane) {
    return plane == 0 ? v[0] : (plane == 1 ? v[1] : v[2]);
}

// ---- records ------------------------------------------------------------------------------
// A group's 4 records live in ONE VGPR: lane l holds dword (l >> 2) & 7 of MB l & 3 (lanes
// 32-63 repeat 0-31).  Per-lane fields of a lane's own MB come out with one ds_bpermute,
// wave-uniform fields with v_readlane.  Loading it is one coalesced global_load_dword, issued
// two groups ahead.
// MP2VG_REC_NT (round 5 A/B): records and coefficient words, read once by one CU, loaded
// nontemporal (streaming) so that they do not displace reference tiles from L2
#ifndef MP2VG_REC_NT
#define MP2VG_REC_NT 0
#endif
__device__ __forceinline__ uint32_t ld_rec(const uint32_t* p) {
    if (MP2VG_REC_NT) return __builtin_nontemporal_load(p);
    return *p;
}
__device__ __forceinline__ uint32_t rec_load(const uint32_t* __restrict__ mbrec, uint32_t g, uint32_t mb_last, int lane) {
    const uint32_t mb = min(g + (uint32_t)(lane & 3), mb_last);
    return ld_rec(&mbrec[(size_t)mb * 8 + ((lane >> 2) & 7)]);
}
__device__ __forceinline__ uint32_t rec_get(uint32_t rv, int f, int k) {  // lane-varying f, k
    return (uint32_t)__builtin_amdgcn_ds_bpermute((f * 4 + k) * 4, (int)rv);
}
template <int F, int K>
__device__ __forceinline__ uint32_t rec_uni(uint32_t rv) {
    return (uint32_t)__builtin_amdgcn_readlane((int)rv, F * 4 + K);
}

// Wave-uniform per-group state (SGPRs), packed so two groups' states fit the SGPR budget.
// Per-lane selection of MB k (lane-varying) is one v_bfe_u32 for byte fields.
struct Group {
    uint32_t fl8;           // byte k: flags & 0xff of MB k (INTRA, DCT_FIELD are used); INTRA if absent
    uint32_t qs8;           // byte k: quantiser_scale
    uint32_t sb8;           // byte k: first coded-block slot of MB k in the group
    uint32_t cbp01, cbp23;  // 16-bit coded_block_pattern of MBs 0,1 / 2,3 (0 if absent)
    int nslots, ncoef;
    uint32_t coef0;
};

__device__ __forceinline__ uint32_t pick8(uint32_t v, int k) { return __builtin_amdgcn_ubfe(v, (uint32_t)k * 8, 8); }
__device__ __forceinline__ uint32_t pick16(uint32_t lo, uint32_t hi, int k) {
    return __builtin_amdgcn_ubfe((k & 2) ? hi : lo, (uint32_t)(k & 1) * 16, 16);
}

template <int NB, int K>
__device__ __forceinline__ void group_mb(Group& S, uint32_t rv, int ng, int& sb, int& cr) {
    const uint32_t r1 = rec_uni<1, K>(rv), r2 = rec_uni<2, K>(rv);
    const bool live = K < ng;
    const uint32_t cbpk = live ? ((r1 >> 16) & ((1u << NB) - 1)) : 0u;
    S.fl8 |= (live ? (r1 & 0xff) : (uint32_t)MP2VG_MB_INTRA) << (8 * K);
    S.qs8 |= (r2 & 0xff) << (8 * K);
    S.sb8 |= (uint32_t)sb << (8 * K);
    if (K == 0) S.cbp01 = cbpk;
    if (K == 1) S.cbp01 |= cbpk << 16;
    if (K == 2) S.cbp23 = cbpk;
    if (K == 3) S.cbp23 |= cbpk << 16;
    sb += __builtin_popcount(cbpk);
    cr += live ? (int)(r2 >> 16) : 0;
}

template <int NB>
__device__ __forceinline__ Group group_state(uint32_t rv, int ng) {
    Group S;
    S.fl8 = S.qs8 = S.sb8 = 0;
    int sb = 0, cr = 0;
    group_mb<NB, 0>(S, rv, ng, sb, cr);
    group_mb<NB, 1>(S, rv, ng, sb, cr);
    group_mb<NB, 2>(S, rv, ng, sb, cr);
    group_mb<NB, 3>(S, rv, ng, sb, cr);
    S.nslots = sb;
    S.ncoef = cr;
    S.coef0 = rec_uni<3, 0>(rv);
    return S;
}

// Pixel-row passes of a group: pass 0 = the 64 luma rows (4 MBs x 16); 4:2:0 pass 1 = Cb + Cr
// (4 x 8 each); 4:2:2 / 4:4:4 pass 1 = Cb, pass 2 = Cr (4 x 16 each).  Rows of the same pixel
// row of adjacent MBs sit in adjacent lanes; a lane's MB is k = lane & 3 in every pass and its
// field-MC vector r = py & 1 = (lane >> 2) & 1.
template <int CF>
struct Passes {
    static constexpr int N = CF == 1 ? 2 : 3;
};
template <int CF, int J>
__device__ __forceinline__ void pass_row(int lane, int& k, int& plane, int& py) {
    k = lane & 3;
    py = lane >> 2;
    if (J == 0) {
        plane = 0;
    } else if (CF == 1) {
        plane = 1 + (lane >> 5);
        py = (lane & 31) >> 2;
    } else {
        plane = J;
    }
}

// ---- anchor tiles ---------------------------------------------------------------------------
// The taps read reference pictures (I and P: the anchors) from a second, tiled copy that the
// anchor's own store pass writes next to its frame_c rows (the tile slot of frame slot i, plane p
// at 2 * plane_off[p]).  A W-px plane (luma and 4:4:4 chroma: W = 16; 4:2:0 / 4:2:2 chroma: W = 8)
// is cut into 128-B tiles, one cache line each: 4 rows x 32 B (W 16) or 8 rows x 16 B (W 8), tile
// t of a band holding pixels [W t, W t + 2 W) -- its own W pixels and, as an apron, the next
// tile's.  A tap row (W + 1 pixels from the dword-aligned x) therefore lies in one tile row, and
// the 17 rows of a luma tap touch 5-6 lines instead of 17 (profiles/r4/README.md: B launch -21 %).
// Tile (band b, column t) sits at (b * ncol + t) * 128 with ncol = stride / W.
template <int W>  // byte offset, in its tile plane, of pixel (x & ~3, y): the tap's row start
__device__ __forceinline__ uint32_t tile_off(uint32_t x, uint32_t y, uint32_t ncol) {
    if (W == 16) return (mul24_asm(y >> 2, ncol) + (x >> 4)) * 128u + (y & 3u) * 32u + (x & 12u);
    return (mul24_asm(y >> 3, ncol) + (x >> 3)) * 128u + (y & 7u) * 16u + (x & 4u);
}
// the two places of the W-px row segment of MB column mx at row y: its own tile (returned) and,
// at own - 128 + W, the apron of the tile to its left
template <int W>
__device__ __forceinline__ uint32_t tile_row(uint32_t mx, uint32_t y, uint32_t ncol) {
    if (W == 16) return (mul24_asm(y >> 2, ncol) + mx) * 128u + (y & 3u) * 32u;
    return (mul24_asm(y >> 3, ncol) + mx) * 128u + (y & 7u) * 16u;
}

// ---- motion compensation taps ---------------------------------------------------------------
// One prediction direction of one pixel row: NW+1 raw dwords of reference row Y from the
// dword-aligned x, loaded one group ahead.  The second row of a vertical half-pel average
// (Y + 1, or Y + 2 for field MC) is the first row of the lane holding the MB's next pixel row
// (lane + 4 / + 8), fetched with ds_bpermute; only a lane on the MB's last row (last two for
// field MC) loads it.  Loads are branch-free (unused taps read the sink) so the compiler's
// in-order vmcnt waits never cover the previous group's stores.
template <int NW>  // output dwords: 4 (16-px row) or 2 (8-px row)
struct Tap {
    static constexpr int ND = NW + 1;
    uint32_t a[ND], b[ND];
    uint32_t ctl;  // bits 0-1 byte shift, 2 half-pel x, 3 half-pel y, 4 used, 5 edge row, 6 field
};

// Reference rows are read with raw buffer loads: the slot base sits in a wave-uniform buffer
// resource (SGPRs) and each lane supplies a 32-bit offset, one VGPR per address.  Offsets at or
// past num_records (= the slot size) return 0 without a memory access: unused taps use kNoTap.
typedef uint32_t u3v __attribute__((ext_vector_type(3)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
constexpr uint32_t kNoTap = 0xFFFFFF00u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slot_rsrc(const uint8_t* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);  // gfx9 raw buffer
}
template <int NW, int ABL = 0>
__device__ __forceinline__ void load_row(uint32_t (&d)[NW + 1], __amdgpu_buffer_rsrc_t r, uint32_t off) {
    if (NW == 4) {
        const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        // (dev ablation 128: no 17th-pixel dword)
        d[4] = __builtin_amdgcn_raw_buffer_load_b32(r, (ABL & 128) ? (int)kNoTap : (int)(off + 16), 0, 0);
    } else if (NW == 2) {
        const u3v v = __builtin_amdgcn_raw_buffer_load_b96(r, (int)off, 0, 0);
        d[0] = v.x; d[1] = v.y; d[2] = v.z;
    } else {
#pragma unroll
        for (int i = 0; i < NW + 1; i++) d[i] = __builtin_amdgcn_raw_buffer_load_b32(r, (int)(off + 4 * i), 0, 0);
    }
}

#ifndef MP2VG_CHROMA_TILES
#define MP2VG_CHROMA_TILES 1
#endif
constexpr bool kChromaTiles = MP2VG_CHROMA_TILES;  // dev A/B: 0 = chroma taps from the frame rows

// v_mad_u32_u24 with a wave-uniform (SGPR) factor: a * b + c, 24-bit a and b (full 32-bit c)
__device__ __forceinline__ uint32_t mad24s_asm(uint32_t a, uint32_t b_uniform, uint32_t c) {
    uint32_t r;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b_uniform), "v"(c));
    return r;
}

// Tap issue (round 6, same-box A/B in profiles/r6/README.md):
// MP2VG_TAP_MAD -- a tap row's tile offset as one 24-bit multiply-add, tile_off(x, y) =
//   (y >> lr) * (ncol * 128 - 128) + y * RB + xterm (RB = 128 >> lr bytes per tile row, xterm =
//   (x >> lw) * 128 + (x & (W - 4)) shared by both rows of the tap): -36 fast, +8 slow VALU per B group;
// MP2VG_ROW2_LOAD -- in the B loop every lane loads its second half-pel row itself (the lane's own
//   row again without vertical half-pel) instead of taking it from the next-row lane by
//   ds_bpermute (-16 ds_bpermute and -48 slow VALU per B group, one more full-width load per
//   direction and pass); the P loop keeps the ds_bpermute (its one direction's TA cost weighs more:
//   +0.5-1 % on the P launch with ROW2).  Both: B launch -3 %, P+B -1 % (c2, one stream), but the
//   two-stream step was neutral or slower on 2 of 3 boxes (profiles/r6/README.md §2): off by default.
#ifndef MP2VG_TAP_MAD
#define MP2VG_TAP_MAD 1
#endif
#ifndef MP2VG_ROW2_LOAD
#define MP2VG_ROW2_LOAD 0
#endif

template <int CF, int NW, int ABL = 0, bool TL = true, bool R2 = false>
__device__ __forceinline__ void tap_issue(Tap<NW>& t, bool use, __amdgpu_buffer_rsrc_t ref, uint32_t plane_off,
                                          uint32_t mvw, int plane, int gx, int py, int phm, int mby_base, bool field,
                                          int fs, int stride, int ph) {
    int mvx = (short)(mvw & 0xffff), mvy = (short)(mvw >> 16);
    if (plane > 0) {  // apply_chroma_scale (mb_decoder.cpp:198-206): arithmetic shift
        if (CF < 3) mvx >>= 1;
        if (CF < 2) mvy >>= 1;
    }
    const int X = gx + (mvx >> 1);
    int Y, step;
    if (!field) {
        Y = mby_base + py + (mvy >> 1);
        step = 1;
    } else {  // field MC (mb_decoder.cpp:229-236): rows 2q + field_select
        Y = mby_base + fs + 2 * ((py >> 1) + (mvy >> 1));
        step = 2;
    }
    // no clamp into the plane: mp2vg_batch_upload refuses any vector whose reads leave the
    // reference planes (the reference's own input contract), and a row offset out of the slot
    // still cannot fault -- the buffer resource returns 0 past num_records
    const int Xc = X;
    const int Y0 = Y;
    const int Y1 = Y + step;
    const int hx = mvx & 1, hy = mvy & 1;
    const bool edge = py + step >= phm;
    t.ctl = (uint32_t)((Xc & 3) | (hx << 2) | (hy << 3) | ((int)use << 4) | ((int)edge << 5) | ((int)field << 6));
    // the rows come from the reference's anchor tiles (tile_off), from the dword-aligned x:
    // byte-exact (unaligned) buffer loads would save two alignbytes per dword but cost twice the
    // texture-address cycles, a net loss (tools/unaligned_check.hip)
    const uint32_t ncol = (uint32_t)stride >> (NW == 4 ? 4 : 3);
    constexpr int LW = NW == 4 ? 4 : 3, LR = NW == 4 ? 2 : 3;  // log2 tile width (px), rows per tile
    const uint32_t xterm = ((uint32_t)Xc >> LW) * 128u + ((uint32_t)Xc & (4u * NW - 4u)) + plane_off;
    const uint32_t pitch_m = ncol * 128u - 128u;  // wave-uniform (issue_pass)
    auto toff = [&](int y) -> uint32_t {
        if (TL && MP2VG_TAP_MAD)
            return mad24s_asm((uint32_t)y >> LR, pitch_m, ((uint32_t)y << (7 - LR)) + xterm);
        return TL ? plane_off + tile_off<4 * NW>((uint32_t)Xc, (uint32_t)y, ncol)
                  : plane_off + (uint32_t)(Xc & ~3) + mul24_asm((uint32_t)y, (uint32_t)stride);
    };
    uint32_t o0 = (use && !(ABL & 32)) ? toff(Y0) : kNoTap;
    // second row: only edge lanes load it (the others take it from the next-row lane, tap_rows),
    // or with MP2VG_ROW2_LOAD every lane (its own row again without vertical half-pel)
    uint32_t o1 = R2 ? ((use && !(ABL & 32)) ? (hy ? toff(Y1) : o0) : kNoTap)
                     : ((use && hy && edge && !(ABL & 32)) ? toff(Y1) : kNoTap);
    if (ABL & 2048) {  // dev ablation (timing only): every tap inside a 64-KB window (L1/L2 hits)
        o0 = o0 == kNoTap ? kNoTap : (o0 & 0xFFFFu);
        o1 = o1 == kNoTap ? kNoTap : (o1 & 0xFFFFu);
    }
    load_row<NW, ABL>(t.a, ref, o0);
    if (!(ABL & 512)) load_row<NW, ABL>(t.b, ref, o1);  // (dev ablation 512: no edge-row loads)
    else for (int i = 0; i <= NW; i++) t.b[i] = 0;
}

// second rows from the next-row lanes (all lanes active: called outside divergent code)
template <int NW>
__device__ __forceinline__ void tap_rows(Tap<NW>& t, int lane) {
    // no vertical half-pel: the second row is the lane's own (avg(r, r) == r, no select later)
    const bool hy = t.ctl & 8;
    const int src = hy ? ((lane + ((t.ctl & 64) ? 8 : 4)) & 63) * 4 : lane * 4;
    const bool edge = hy && (t.ctl & 32);
#pragma unroll
    for (int i = 0; i <= NW; i++) {
        const uint32_t nb = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)t.a[i]);
        t.b[i] = edge ? t.b[i] : nb;
    }
}

// cascaded half-pel average of one row (mc_sse2.hpp:5-39 == mc_c.hpp:15), branch-free:
// alignbyte by hx (0 or 1) yields the x+1 pixels or the row itself, and avg(x, x) == x (the
// second row of a lane without vertical half-pel is its own row, see tap_rows).
template <int NW>
__device__ __forceinline__ void tap_finish(const Tap<NW>& t, uint32_t (&p)[NW]) {
    const uint32_t s = t.ctl & 3, hx = (t.ctl >> 2) & 1;
    uint32_t A[NW + 1], C[NW + 1];
#pragma unroll
    for (int d = 0; d < NW; d++) {
        A[d] = __builtin_amdgcn_alignbyte(t.a[d + 1], t.a[d], s);
        C[d] = __builtin_amdgcn_alignbyte(t.b[d + 1], t.b[d], s);
    }
    A[NW] = t.a[NW] >> (8 * s);  // only its byte 0 is used (the 17th / 9th pixel)
    C[NW] = t.b[NW] >> (8 * s);
#pragma unroll
    for (int d = 0; d < NW; d++) {
        const uint32_t r0 = avg4(A[d], __builtin_amdgcn_alignbyte(A[d + 1], A[d], hx));
        const uint32_t r1 = avg4(C[d], __builtin_amdgcn_alignbyte(C[d + 1], C[d], hx));
        p[d] = avg4(r0, r1);
    }
}

// prediction of one pass: forward / backward / their average (mc_sse2.hpp:78-84); 0 for intra.
// MCM: 1 = forward only (P pictures), 2 = both directions (B pictures).
template <int MCM, int NW, int ABL = 0>
__device__ __forceinline__ void predict(Tap<NW>& tf, Tap<NW>& tb, int lane, uint32_t (&p)[NW]) {
    if (ABL & 64) {  // dev ablation: no prediction arithmetic
#pragma unroll
        for (int d = 0; d < NW; d++) p[d] = tf.a[d] ^ tf.b[d] ^ (MCM == 2 ? tb.a[d] ^ tb.b[d] : 0u);
        return;
    }
    if (!(MP2VG_ROW2_LOAD && MCM == 2)) {  // (ROW2: the B loop's taps loaded both rows)
        tap_rows<NW>(tf, lane);
        if (MCM == 2) tap_rows<NW>(tb, lane);
    }
    const bool uf = tf.ctl & 16, ub = MCM == 2 && (tb.ctl & 16);
    uint32_t pf[NW], pb[NW];
#pragma unroll
    for (int d = 0; d < NW; d++) pf[d] = pb[d] = 0;
    if (uf) tap_finish<NW>(tf, pf);
    if (MCM == 2 && ub) tap_finish<NW>(tb, pb);
#pragma unroll
    for (int d = 0; d < NW; d++) p[d] = (uf && ub) ? avg4(pf[d], pb[d]) : (uf ? pf[d] : pb[d]);
}

// per-lane record fields of the lane's MB that the tap issue needs
struct LaneRec {
    uint32_t r0, r1, mvf, mvb;
};
__device__ __forceinline__ LaneRec lane_rec(uint32_t rv, int lane) {
    LaneRec L;
    const int k = lane & 3;
    L.r0 = rec_get(rv, 0, k);
    L.r1 = rec_get(rv, 1, k);
    const int r = (L.r1 & MP2VG_MB_FIELD_MC) ? ((lane >> 2) & 1) : 0;
    L.mvf = rec_get(rv, 4 + 2 * r, k);  // mv[r][0]
    L.mvb = rec_get(rv, 5 + 2 * r, k);  // mv[r][1]
    return L;
}

// MCM 1 (the one-reference loop: P pictures, and B pictures that predict in one direction only,
// runtime.cpp plan_batch): every non-intra MB predicts from ref_fwd, with its forward (dir 0) or
// backward (dir 1: ref_fwd then holds the backward reference) vectors and field selects.
template <int CF, int MCM, int J, int NW, int ABL = 0>
__device__ __forceinline__ void issue_pass(const LaneRec& L, bool live, int lane, const Geo& geo,
                                           __amdgpu_buffer_rsrc_t ref_fwd, __amdgpu_buffer_rsrc_t ref_bwd,
                                           Tap<NW>& tf, Tap<NW>& tb, int dir = 0) {
    using F = Fmt<CF>;
    int k, plane, py;
    pass_row<CF, J>(lane, k, plane, py);
    const uint32_t fl = L.r1 & 0xffff;
    const bool none = !live || (fl & MP2VG_MB_INTRA);
    const bool bwd = fl & MP2VG_MB_BWD;
    const bool fwd = !none && (MCM == 1 || (fl & MP2VG_MB_FWD) || !bwd);
    const bool field = fl & MP2VG_MB_FIELD_MC;
    const int pw = plane == 0 ? 16 : F::CW;
    const int phm = plane == 0 ? 16 : F::CH;
    const int gx = (int)(L.r0 & 0xffff) * pw;
    const int mbyb = (int)(L.r0 >> 16) * phm;
    const int r = field ? (py & 1) : 0;
    // wave-uniform: a pass is luma (J 0) or chroma, and Cb and Cr share their stride and height
    // (frame_c layout), so the row pitch stays in SGPRs (lane-selected, it cost readfirstlanes)
    const int stride = J == 0 ? geo.stride[0] : geo.stride[1];
    const int ph = J == 0 ? geo.ph[0] : geo.ph[1];
    constexpr bool TL = J == 0 || kChromaTiles;
    const uint32_t off = (TL ? 2u : 1u) * (uint32_t)gsel(geo.plane_off, plane);  // the plane in the tile slot
    const uint32_t mv1 = (MCM == 1 && dir) ? L.mvb : L.mvf;
    const int fsh = 8 + 2 * r + (MCM == 1 ? dir : 0);
    constexpr bool R2 = MP2VG_ROW2_LOAD && MCM == 2;
    tap_issue<CF, NW, ABL, TL, R2>(tf, fwd, ref_fwd, off, mv1, plane, gx, py, phm, mbyb, field, (fl >> fsh) & 1, stride, ph);
    if (MCM == 2)
        tap_issue<CF, NW, ABL, TL, R2>(tb, !none && bwd, ref_bwd, off, L.mvb, plane, gx, py, phm, mbyb, field,
                                       (fl >> (9 + 2 * r)) & 1, stride, ph);
}

// frame_c row stores (16 / 8 B).  Nontemporal stores measured c2 -8.5 %, c3 -19 % (round 4).
__device__ __forceinline__ void row_store16(uint8_t* d, uint32_t a, uint32_t b, uint32_t c, uint32_t e) {
    *(uint4*)d = make_uint4(a, b, c, e);
}
__device__ __forceinline__ void row_store8(uint8_t* d, uint32_t a, uint32_t b) { *(uint2*)d = make_uint2(a, b); }

// Cache policy of the frame-row and anchor-tile stores: 0 = plain global stores; otherwise
// buffer stores through the slot's resource with these aux bits (gfx950: 1 sc0, 2 nt, 16 sc1),
// dead lanes at an out-of-range offset (the store is discarded).  Measured, c2, two boxes, same-box
// arms interleaved (profiles/r5/README.md):
//   tiles nt (streaming: the lines stay in L2 but go first)  +4.0-4.8 %  (the I launch -10-13 %)
//   tiles sc1 (write through, line dropped from L2)           -0.2 %
//   tiles nt + sc1                                            +1.6 %
//   rows sc1 (write-through: no later recon launch reads the   +1.5 % alone, +0.5 % over tiles nt
//            frame_c rows -- the taps read the tiles -- but tile_convert (after a mode-4 I launch,
//            for B pictures read later, for invalidated slots), digest_kernel and the drop-in's
//            frame_copy_kernel do, after the launch boundary; the A/B covers the c2 P/B path)
//   rows nt                                                   -3.5 % over tiles nt
//   records + coefficient words nt loads                      -0.5 %
#ifndef MP2VG_ROW_POL
#define MP2VG_ROW_POL 16
#endif
#ifndef MP2VG_TILE_POL
#define MP2VG_TILE_POL 2
#endif
template <int POL>
__device__ __forceinline__ void pol_store16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(u4v{v.x, v.y, v.z, v.w}, r, (int)off, 0, POL);
}
template <int POL>
__device__ __forceinline__ void pol_store8(__amdgpu_buffer_rsrc_t r, uint32_t off, uint2 v) {
    typedef uint32_t u2v __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(u2v{v.x, v.y}, r, (int)off, 0, POL);
}

// ---- add/clip + store ----------------------------------------------------------------------

// tiles (uniform: the picture is read by a later one, runtime.cpp TilePlan): the row's pixels
// also go over the first half of its int16 residual row in LDS, from which tile_group writes the
// picture's anchor tiles in whole lines
template <int CF, int J, int NW, int ABL>
__device__ __forceinline__ void store_pass(uint32_t r0, uint32_t r1, bool live, int lane, const Geo& geo, uint8_t* wsink,
                                           uint8_t* dst_slot, __amdgpu_buffer_rsrc_t dst_rsrc, bool tiles,
                                           const short* s_res_wave, const uint32_t (&p)[NW]) {
    using F = Fmt<CF>;
    using RL = ResLayout<CF>;
    int k, plane, py;
    pass_row<CF, J>(lane, k, plane, py);
    const uint32_t fl = r1 & 0xffff, cbpk = r1 >> 16;
    // put: packus(res); add: packus(adds(pred, res))   (idct_sse2.hpp:106-119)
    const int lb = left_block<CF>(plane, py, fl & MP2VG_MB_DCT_FIELD);
    const int rb = (plane == 0) ? lb + 1 : lb + 4;
    const bool cl = cbpk & (1u << lb);
    const bool cr = NW == 4 && (cbpk & (1u << rb));
    uint32_t out[4] = {0, 0, 0, 0};
#pragma unroll
    for (int d = 0; d < NW; d++) out[d] = p[d];
    if (cl || cr) {
        const short* res = s_res_wave + k * RL::MBS + RL::base(plane) + py * RL::width(plane);
        uint32_t rv[8];
        const uint4 q0 = *(const uint4*)&res[0];
        rv[0] = q0.x; rv[1] = q0.y; rv[2] = q0.z; rv[3] = q0.w;
        if (NW == 4) {
            const uint4 q1 = *(const uint4*)&res[8];
            rv[4] = q1.x; rv[5] = q1.y; rv[6] = q1.z; rv[7] = q1.w;
        }
#pragma unroll
        for (int d = 0; d < NW; d++) {
            if (!(d < 2 ? cl : cr)) continue;
            // pairs (x0, x0+2) and (x0+1, x0+3) as packed i16
            const uint32_t lo = __builtin_amdgcn_perm(0u, out[d], 0x0c020c00u);
            const uint32_t hi = __builtin_amdgcn_perm(0u, out[d], 0x0c030c01u);
            const short2_t a = __builtin_bit_cast(short2_t, lo) + __builtin_bit_cast(short2_t, rv[2 * d]);
            const short2_t c = __builtin_bit_cast(short2_t, hi) + __builtin_bit_cast(short2_t, rv[2 * d + 1]);
            // packus: bytes x0 = a.lo, x0+1 = c.lo, x0+2 = a.hi, x0+3 = c.hi
            out[d] = __builtin_amdgcn_perm(sat_pk_u8(c), sat_pk_u8(a), 0x05010400u);
        }
    }
    const int pw = plane == 0 ? 16 : F::CW;
    const int phm = plane == 0 ? 16 : F::CH;
    const uint32_t doff = gsel(geo.plane_off, plane) + mul24_asm((r0 >> 16) * phm + py, (uint32_t)gsel(geo.stride, plane)) +
                          (r0 & 0xffff) * (uint32_t)pw;
    uint8_t* dst = dst_slot + doff;
    dst = live ? dst : wsink;  // branch-free: every lane stores (see Tap)
    if (ABL & 8192)  // dev ablation (timing only): each store instruction writes 1 KB contiguous
        dst = dst_slot + ((((r0 & 0xffff) + (r0 >> 16) * 128u) * 3u + (uint32_t)J) * 1024u + (uint32_t)lane * 16u) %
                             (uint32_t)(geo.plane_off[1] - 1024);
    if (tiles) {  // the row's pixels for tile_group: over the first half of its (read) int16 residual row
        uint8_t* img = (uint8_t*)(s_res_wave + k * RL::MBS + RL::base(plane) + py * RL::width(plane));
        if (NW == 4)
            *(uint4*)img = make_uint4(out[0], out[1], out[2], out[3]);
        else
            *(uint2*)img = make_uint2(out[0], out[1]);
    }
    if (ABL & 8) {
        asm volatile("" ::"v"(out[0]), "v"(out[1]), "v"(out[2]), "v"(out[3]), "v"(dst));
    } else if (ABL & 4096) {  // dev ablation (timing only): one dword per row store (1/4, 1/2 bytes)
        asm volatile("" ::"v"(out[0]), "v"(out[1]), "v"(out[2]), "v"(out[3]));
        *(uint32_t*)dst = out[0] ^ out[1] ^ (NW == 4 ? out[2] ^ out[3] : 0u);
    } else if (MP2VG_ROW_POL != 0) {
        if (NW == 4)
            pol_store16<MP2VG_ROW_POL>(dst_rsrc, live ? doff : kNoTap, make_uint4(out[0], out[1], out[2], out[3]));
        else
            pol_store8<MP2VG_ROW_POL>(dst_rsrc, live ? doff : kNoTap, make_uint2(out[0], out[1]));
    } else if (NW == 4) {
        row_store16(dst, out[0], out[1], out[2], out[3]);
    } else {
        row_store8(dst, out[0], out[1]);
    }
}

// C8 (I kernels): the row's clamped pixels from the byte residual image, reordered from the
// ResLayout order (x0, x0+2, x0+1, x0+3 in each 4-pixel group) by one v_perm per dword
template <int CF, int J, int NW>
__device__ __forceinline__ void store_pass_put8(uint32_t r0, bool live, int lane, const Geo& geo, uint8_t* wsink,
                                                uint8_t* dst_slot, __amdgpu_buffer_rsrc_t dst_rsrc,
                                                const uint8_t* res8_wave) {
    using F = Fmt<CF>;
    using RL = ResLayout<CF>;
    int k, plane, py;
    pass_row<CF, J>(lane, k, plane, py);
    const uint8_t* row = &res8_wave[k * RL::SIZE + RL::base(plane) + py * RL::width(plane)];
    const int pw = plane == 0 ? 16 : F::CW;
    const int phm = plane == 0 ? 16 : F::CH;
    const uint32_t doff = gsel(geo.plane_off, plane) + mul24_asm((r0 >> 16) * phm + py, (uint32_t)gsel(geo.stride, plane)) +
                          (r0 & 0xffff) * (uint32_t)pw;
    uint8_t* dst = live ? dst_slot + doff : wsink;  // branch-free: every lane stores (see Tap)
    if (NW == 4) {
        const uint4 q = *(const uint4*)row;
        const uint4 o = make_uint4(__builtin_amdgcn_perm(q.x, q.x, 0x03010200u), __builtin_amdgcn_perm(q.y, q.y, 0x03010200u),
                                   __builtin_amdgcn_perm(q.z, q.z, 0x03010200u), __builtin_amdgcn_perm(q.w, q.w, 0x03010200u));
        if (MP2VG_ROW_POL != 0)
            pol_store16<MP2VG_ROW_POL>(dst_rsrc, live ? doff : kNoTap, o);
        else
            row_store16(dst, o.x, o.y, o.z, o.w);
    } else {
        const uint2 q = *(const uint2*)row;
        const uint2 o = make_uint2(__builtin_amdgcn_perm(q.x, q.x, 0x03010200u), __builtin_amdgcn_perm(q.y, q.y, 0x03010200u));
        if (MP2VG_ROW_POL != 0)
            pol_store8<MP2VG_ROW_POL>(dst_rsrc, live ? doff : kNoTap, o);
        else
            row_store8(dst, o.x, o.y);
    }
}

// The group's anchor tiles, written in whole tile lines from LDS (I kernels: the byte residual
// image; P loops: the pixels store_pass left in the residual image).
// A group of 4 MBs (columns t0..t0+3) owns tiles t0..t0+2 of each band completely and two half
// tiles: t0+3's own half (MB 3) and t0-1's apron half (MB 0; none at column 0).  Unit u of a
// W-16 plane: u < 96 -> tile t0 + (u >> 5), band (u >> 3) & 3 of the MB row, chunk u & 7 (row
// chunk >> 1, half chunk & 1: MB j + half), so 8 consecutive lanes fill one 128-B line; 96..127 ->
// the half tiles' 16-B rows.  A W-8 plane (4:2:0 / 4:2:2 chroma): 16-B units are whole tile rows
// [MB j row | MB j+1 row] of tiles t0..t0+2, 8-B units the half tiles' rows.  Row stores of the
// same bytes (one row per lane, own and apron place) left 16-B pieces 32 B apart in every line:
// I launch +35-60 % instead of +30 % (profiles/r4/README.md).
// a row of the group's pixels from LDS: the I kernels' byte residual image (compact layout, each
// dword in the x0, x0+2, x0+1, x0+3 order of ResLayout: one v_perm); P/B kernels (NAT): the
// final pixels in natural order that store_pass left in the first half of each int16 residual row
template <int CF, bool NAT>
__device__ __forceinline__ const uint8_t* img_row(const uint8_t* img, int k, int plane, int py) {
    using RL = ResLayout<CF>;
    return &img[(NAT ? 2 : 1) * (k * (NAT ? RL::MBS : RL::SIZE) + RL::base(plane) + py * RL::width(plane))];
}
__device__ __forceinline__ uint32_t unswz(uint32_t v, bool nat) { return nat ? v : __builtin_amdgcn_perm(v, v, 0x03010200u); }
template <int CF, bool NAT>
__device__ __forceinline__ uint4 img_row16(const uint8_t* img, int k, int plane, int py) {
    const uint4 q = *(const uint4*)img_row<CF, NAT>(img, k, plane, py);
    return make_uint4(unswz(q.x, NAT), unswz(q.y, NAT), unswz(q.z, NAT), unswz(q.w, NAT));
}
template <int CF, bool NAT>
__device__ __forceinline__ uint2 img_row8(const uint8_t* img, int k, int plane, int py) {
    const uint2 q = *(const uint2*)img_row<CF, NAT>(img, k, plane, py);
    return make_uint2(unswz(q.x, NAT), unswz(q.y, NAT));
}
template <int CF, bool NAT, int ABL = 0>
__device__ __forceinline__ void tile_group(uint32_t mx0, uint32_t mby, int lane, const Geo& geo, uint8_t* wsink,
                                           uint8_t* dst_tiles, __amdgpu_buffer_rsrc_t tile_rsrc, const uint8_t* res8) {
    using F = Fmt<CF>;
    constexpr bool POL = MP2VG_TILE_POL != 0;
    // W-16 planes: luma, and the 4:4:4 chroma planes
    for (int plane = 0; plane < (CF == 3 && kChromaTiles ? 3 : 1); plane++) {
        uint8_t* tp = dst_tiles + 2u * gsel(geo.plane_off, plane);
        const uint32_t ncol = (uint32_t)gsel(geo.stride, plane) >> 4;
#pragma nounroll
        for (int i = 0; i < 2; i++) {
            const int u = lane + 64 * i;
            int j, r, h;
            if (u < 96) {
                j = u >> 5, r = ((u >> 3) & 3) * 4 + ((u & 7) >> 1), h = u & 1;
            } else {
                const int side = (u - 96) >> 4;
                r = u & 15, h = side, j = side ? -1 : 3;
            }
            const uint4 v = img_row16<CF, NAT>(res8, j + h, plane, r);
            const bool none = j < 0 && mx0 == 0;
            const uint32_t o = tile_row<16>(mx0 + (uint32_t)j, mby * 16u + (uint32_t)r, ncol) + (uint32_t)h * 16u;
            if (POL)
                pol_store16<MP2VG_TILE_POL>(tile_rsrc, none ? kNoTap : 2u * gsel(geo.plane_off, plane) + o, v);
            else
                *(uint4*)(none ? wsink : ((ABL & 65536) ? dst_tiles + (o & 0xFFF0u) : tp + o)) = v;
        }
    }
    if constexpr (CF != 3 && kChromaTiles) {  // W-8 chroma: Cb and Cr
        constexpr int RPM = F::CH;  // chroma rows per MB (8 or 16)
        constexpr int N16 = 2 * 3 * RPM, N8 = 2 * 2 * RPM;
        const uint32_t ncol = (uint32_t)geo.stride[1] >> 3;
#pragma nounroll
        for (int i = 0; i < (N16 + 63) / 64; i++) {
            const int u = lane + 64 * i;
            const int plane = 1 + (u >= 3 * RPM ? 1 : 0), rem = u - (plane - 1) * 3 * RPM;
            const int j = rem / RPM, r = rem % RPM;
            const uint2 a = img_row8<CF, NAT>(res8, j, plane, r), b = img_row8<CF, NAT>(res8, min(j + 1, 3), plane, r);
            const uint32_t o = tile_row<8>(mx0 + (uint32_t)j, mby * (uint32_t)RPM + (uint32_t)r, ncol);
            if (POL) {
                pol_store16<MP2VG_TILE_POL>(tile_rsrc, u < N16 ? 2u * gsel(geo.plane_off, plane) + o : kNoTap,
                                            make_uint4(a.x, a.y, b.x, b.y));
            } else {
                uint8_t* d = (ABL & 65536) ? dst_tiles + (o & 0xFFF0u) : dst_tiles + 2u * gsel(geo.plane_off, plane) + o;
                *(uint4*)(u < N16 ? d : wsink) = make_uint4(a.x, a.y, b.x, b.y);
            }
        }
#pragma nounroll
        for (int i = 0; i < (N8 + 63) / 64; i++) {
            const int u = lane + 64 * i;
            const int plane = 1 + (u >= 2 * RPM ? 1 : 0), rem = u - (plane - 1) * 2 * RPM;
            const int side = rem / RPM, r = rem % RPM;
            const int j = side ? -1 : 3, h = side;
            const uint2 v = img_row8<CF, NAT>(res8, side ? 0 : 3, plane, r);
            const uint32_t o = tile_row<8>(mx0 + (uint32_t)j, mby * (uint32_t)RPM + (uint32_t)r, ncol) + (uint32_t)h * 8u;
            const bool none = u >= N8 || (side && mx0 == 0);
            if (POL) {
                pol_store8<MP2VG_TILE_POL>(tile_rsrc, none ? kNoTap : 2u * gsel(geo.plane_off, plane) + o, v);
            } else {
                uint8_t* d = (ABL & 65536) ? dst_tiles + (o & 0xFFF8u) : dst_tiles + 2u * gsel(geo.plane_off, plane) + o;
                *(uint2*)(none ? wsink : d) = v;
            }
        }
    }
}

// ---- one slice ------------------------------------------------------------------------------
// Slices per workgroup (`mates`, recon_kernel): 2 or 4 cluster-mate slices in the 4-wave P/B
// kernels, at most as many as the LDS holds matrix sets (Lds::NH: 4, or 2 in 4:4:4); 1 otherwise.
// The one rule for the host's grid size (launch_one) and the kernel's slice index.
// dev ablations that keep the I kernels' compact layout: 16 stamps, 32768 none, 65536 tile stores
// into a 64-KB window of the tile slot (L2-resident: the stores' memory traffic, not their issue)
constexpr int kAblCompact = 16 | 32768 | 65536;
template <int MCM, int ABL>
constexpr bool compact_layout() { return (MCM == 0 || MCM == 4) && (ABL & ~kAblCompact) == 0; }
constexpr int lds_sets(int cf, bool c8) { return c8 ? 1 : (cf == 3 ? 2 : 4); }
template <int CF, int MCM, int ABL>
constexpr uint32_t slices_per_wg(uint32_t mates) {
    return !compact_layout<MCM, ABL>() && kernel_waves<MCM, ABL>() == 4 && (mates == 2 || mates == 4) &&
                   mates <= (uint32_t)lds_sets(CF, false)
               ? mates
               : 1u;
}
constexpr int BLKS = 72;
// C8 = the compact layout of the I kernels (4:4:4: 38.4 KB instead of 53.8 KB per workgroup, so
// four workgroups share a CU instead of three; 4:2:2 26.0 KB, 4:2:0 19.9 KB).  (A double-buffered
// P/B layout for a cross-group IDCT pipeline -- pass 1 of group g beside pass 2 of g-1 in shared
// rounds -- was built and measured -7.5 % on c2, profiles/r6/README.md; commit d02a2a6 has it.)
template <int CF, bool C8 = false, int NWV = WAVES>
struct Lds {
    static constexpr bool COMPACT = C8;
    static constexpr bool X64 = C8;              // 128-B block slots, 16-B chunk index XOR (slot & 7)
    static constexpr int NBUF = 1;               // block buffers (and slot maps) per wave
    static constexpr int NWAVES = NWV;           // waves per workgroup
    static constexpr int STEP = NWV * G;         // a wave's next group starts STEP MBs later
    static constexpr int MAXS = G * Fmt<CF>::NB;  // coded-block slots per group
    // coef raster -> pass-1 out.  Slots 144 B apart (BLK = 72 shorts): the transposed pass-1
    // writes of the 8 slots in a 32-lane half then hit distinct banks (128 B apart: 8-way
    // conflicts).  C8: slots 128 B apart with the 16-B chunk index XOR (slot & 7), same banks.
    static constexpr int BLK = X64 ? 64 : BLKS;
    short blk[NWV * NBUF][MAXS][BLK];  // wave w, buffer b: blk[w * NBUF + b]
    // residual images, int16 in ResLayout; C8 (intra only: output = clamp(residual)): the clamped
    // pixels as bytes in the same ResLayout order, half the size
    short res[NWV][C8 ? G * ResLayout<CF>::SIZE / 2 : G * ResLayout<CF>::MBS];
    uint8_t map[NWV * NBUF][MAXS];               // slot -> k*16 + b
    uint32_t dq[NWV][64];                        // (k*16 + b) -> dequant parameters (DqEntry)
    // quantiser matrices and scan (C8: the I kernels' one picture per workgroup; P/B layouts NH
    // sets, one per slice when the workgroup runs several, recon_kernel `mates`; 4:4:4 two, so
    // three workgroups still share a CU)
    static constexpr int NH = lds_sets(CF, C8);
    uint8_t W[4 * NH][64];
    // I kernels (WB): the intra matrix row of each block b (W[0] for b < 6, W[2] above), so a
    // coefficient word's (b, i) bits 16-25 index it directly; scan positions stored doubled (byte
    // offsets of an int16 in the block).  The table sits after `scan`: c5 is sensitive to where
    // the small tables sit (scan 64 B further on: -5 %; the table in front of scan: -1 %)
    static constexpr bool WB = C8;
    uint8_t scan[64 * NH];
    uint8_t Wb[WB && CF != 1 ? Fmt<CF>::NB : 0][64];  // zero-length (clang extension) when unused: no layout change
    // I kernels (MP2VG_I_KBTAB): per coefficient word's (MB in group k, block b) = bits 22-27, the
    // block's byte address in the wave's blocks with its XOR chunk base, slot * 128 | (slot & 7) * 16
    // (bits 8-23), and k * 8, the bit offset of MB k's quantiser scale in qs8 (bits 0-4, which is
    // what v_bfe_u32 reads of its offset operand: no shift per word): one LDS
    // read in place of the slot arithmetic (bfe, bfe, mad, three shifts, bitop3, add3) per word
    // round.  Last in the layout: c5 is sensitive to where the small tables above sit.
    uint32_t kbtab[WB ? 64 : 0];
    // short index of coefficient / pass-1 output idx (0..63) of a slot, relative to the wave's blk
    __device__ static int bofs(int slot, int idx) { return slot * BLK + (X64 ? (idx ^ ((slot & 7) << 3)) : idx); }
};

// (MB in group) * 16 + block of coded-block slot `slot`: from the group's slot map, or, in I
// pictures (every MB intra with every block coded), slot = k * NB + b directly
template <int MCM, int NB, class LT>
__device__ __forceinline__ int slot_kb(const LT& L, int wave, int slot, int buf = 0) {
    if constexpr (MCM == 0) {
        // slot / NB by a 24-bit multiply and a shift, exact for the slots of a group (< 4 * NB)
        // (a plain division became a quarter-rate v_mul_hi_i32 + v_mad_u64_u32)
        static_assert(NB == 6 || NB == 8 || NB == 12, "blocks per MB");
        const int k = NB == 8 ? slot >> 3 : (int)(__umul24((uint32_t)slot, 43u) >> (NB == 6 ? 8 : 9));
        return (k << 4) | (slot - k * NB);
    } else {
        return L.map[wave * LT::NBUF + buf][slot];
    }
}

// IDCT pass 1's transposed writes: the 8 output pairs of lane (slot, v) go to chunk x of the
// slot, element v.  In the compact layout chunk x sits at (x ^ (slot & 7)) * 16 bytes, so with the
// LDS image 128-B aligned (the kernel's only __shared__ object, aligned(128); slots 128 B, wave
// blocks multiples of 128 B) the byte address of chunk x is that of chunk 0 XOR x * 16: one v_xor
// per write instead of an XOR and a shift-add
typedef __attribute__((address_space(3))) short2_t lds_short2_t;
typedef __attribute__((address_space(3))) u4v lds_uint4_t;  // (HIP's uint4 class takes no address space)
__device__ __forceinline__ uint4 ld16(const lds_uint4_t* p) {
    const u4v v = *p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void zero16(lds_uint4_t* p) { *p = u4v{0u, 0u, 0u, 0u}; }
template <class LT>
__device__ __forceinline__ void pass1_store(short* bw, int slot, int v, const short2_t (&s)[8]) {
    if constexpr (LT::X64) {
        const uint32_t b0 = (uint32_t)(uintptr_t)(lds_short2_t*)(bw + LT::bofs(slot, v));  // chunk 0 ^ (slot & 7)
#pragma unroll
        for (int x = 0; x < 8; x++) *(lds_short2_t*)(uintptr_t)(b0 ^ (uint32_t)(x << 4)) = s[x];
    } else {
#pragma unroll
        for (int x = 0; x < 8; x++) *(short2_t*)&bw[LT::bofs(slot, x * 8 + v)] = s[x];
    }
}

// IDCT pass 2's intra put (idct_sse2.hpp:106-108, packus(res >> 6)) of columns (x, x+2) of a
// block: row y at byte address a0 + y * step in the byte residual image.  The row step is
// lane-varying (field DCT), so the address runs by one add per row (the row-index form cost a
// shift-add and an add per row, and the MB offset a quarter-rate multiply)
typedef __attribute__((address_space(3))) uint16_t lds_u16_t;

// 16-B chunks ca, cb (0-7) of coded-block slot `slot` as LDS pointers, computed once for the read
// and pass 2's zeroing (compact layout: chunk 0 XOR 16c, see pass1_store)
template <class LT>
__device__ __forceinline__ void slot_chunks(short* bw, int slot, int ca, int cb, lds_uint4_t*& pa, lds_uint4_t*& pb) {
    if constexpr (LT::X64) {
        const uint32_t b0 = (uint32_t)(uintptr_t)(lds_short2_t*)(bw + LT::bofs(slot, 0));
        pa = (lds_uint4_t*)(uintptr_t)(b0 ^ (uint32_t)(ca << 4));
        pb = (lds_uint4_t*)(uintptr_t)(b0 ^ (uint32_t)(cb << 4));
    } else {
        const uint32_t b0 = (uint32_t)(uintptr_t)(lds_short2_t*)(bw + slot * LT::BLK);
        pa = (lds_uint4_t*)(uintptr_t)(b0 + (uint32_t)(ca << 4));
        pb = (lds_uint4_t*)(uintptr_t)(b0 + (uint32_t)(cb << 4));
    }
}
__device__ __forceinline__ void put8_rows(uint32_t a0, uint32_t step, const short2_t (&s)[8]) {
#pragma unroll
    for (int y = 0; y < 8; y++) *(lds_u16_t*)(uintptr_t)(a0 + (uint32_t)y * step) = (uint16_t)sat_pk_u8(s[y] >> (short)6);
}

struct SliceCtx {
    const uint32_t* mbrec;
    const uint32_t* coefs;
    uint8_t* dst_slot;
    uint8_t* dst_tiles;  // the picture's anchor tiles
    __amdgpu_buffer_rsrc_t dst_rsrc, tile_rsrc;  // the same as buffer resources (store policies)
    bool tiles;          // ... which it writes (SliceDesc.reserved bit 0, runtime.cpp TilePlan)
    int dir;             // MCM 1: 1 = the one reference is the backward one (SliceDesc.reserved bit 2)
    // this wave's own 64-B sink line (dummy and dead-lane stores): stores of many waves to one
    // address serialize in one L2 channel, and a wave's first loop-head wait covers its own
    uint8_t* wsink;
    __amdgpu_buffer_rsrc_t ref_fwd, ref_bwd;
    __amdgpu_buffer_rsrc_t cref_fwd, cref_bwd;  // chroma taps' source (the tiles, or frame rows)
    __amdgpu_buffer_rsrc_t coef_rsrc;  // the batch's words; offsets >= kNoTap read nothing
    uint32_t mb_begin, mb_end;
    // the wave's place among the waves of its slice and their group stride (STEP MBs): 4 waves
    // per slice, or 4 / mates when the workgroup runs `mates` slices (recon_kernel; half = which)
    uint32_t wpos, step;
    int half;
};

// Per-group dequant parameters of block b of MB k, built once per group by lane k*16 + b:
// bits 0-7 coded-block slot, 8-15 quantiser_scale, 16-17 quantiser matrix (W row), 18 intra,
// 19 coded (cbp bit set and b < NB).
template <int CF>
__device__ __forceinline__ uint32_t dq_entry(const Group& S, int lane) {
    constexpr int NB = Fmt<CF>::NB;
    const int k = lane >> 4, bb = lane & 15;
    const uint32_t cbpk = pick16(S.cbp01, S.cbp23, k);
    const bool coded = bb < NB && ((cbpk >> bb) & 1);
    const uint32_t slot = pick8(S.sb8, k) + (uint32_t)__builtin_popcount(cbpk & ((1u << bb) - 1));
    const uint32_t intra = pick8(S.fl8, k) & MP2VG_MB_INTRA;
    const uint32_t wsel = (bb < 6 ? 0u : 2u) + (intra ? 0u : 1u);
    return (slot & 0xff) | (pick8(S.qs8, k) << 8) | (wsel << 16) | (intra << 18) | ((uint32_t)coded << 19);
}

__device__ __forceinline__ int mul24i_asm(int a, int b) {  // v_mul_i32_i24: signed 24 x 24, low 32 bits
    int r;
    asm("v_mul_i32_i24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// dequant of one coefficient word (parse_block, mb_decoder.cpp:74-155) into its coded-block
// slot: lane = word; its MB k (from the word's MB-column bits) and block select the group's
// dequant entry.  INTRA_ONLY (I pictures: every MB intra with every block coded, no '1s' first
// coefficients) needs no table: the slot is k * NB + b, the matrix is the block's (luma for
// blocks 0-5, mb_decoder.cpp:111-113), the quantiser scale is byte k of qs8.
template <class LT, bool INTRA_ONLY = false, int NB = 6>
__device__ __forceinline__ void dequant_word(LT& L, int wave, uint32_t w, uint32_t qs8, bool live = true, int h = 0,
                                             int buf = 0) {
    if constexpr (INTRA_ONLY) {
        const uint32_t k = (w >> 26) & 3u, b = (w >> 22) & 15u;
        const int slot = (int)(k * NB + b);
        const int i = (w >> 16) & 63;
        const int level = (short)(w & 0xffff);
        // 4:2:0: every block uses the luma intra matrix (blocks 4/5 too, mb_decoder.cpp:184-185),
        // so W[0][i] directly: one 64-B table, no bank conflicts between block rows
        const int Wi = NB == 6 ? L.W[4 * h][i]
                               : (LT::WB ? ((const uint8_t*)L.Wb)[(w >> 16) & 0x3ffu] : L.W[4 * h + (b < 6 ? 0 : 2)][i]);
        uint32_t kb = 0;  // the (k, b) table entry (MP2VG_I_KBTAB)
        if constexpr (LT::WB && MP2VG_I_KBTAB) kb = L.kbtab[(w >> 22) & 63u];
        // (v_bfe_u32 reads its offset's low 5 bits: the entry's k * 8)
        const uint32_t qsk = (LT::WB && MP2VG_I_KBTAB) ? __builtin_amdgcn_ubfe(qs8, kb, 8) : pick8(qs8, (int)k);
        const uint32_t wq = __umul24((uint32_t)Wi, qsk);
        // (|level| * W * qs) >> 4 with the sign applied after the shift (truncation toward zero):
        // the signed product, biased by 15 when negative, then an arithmetic shift
        const int p = mul24i_asm(level, (int)wq);
        const int val = (p + ((p >> 31) & 15)) >> 4;
        const int v = min(max((int)(short)val, -2048), 2047);  // int16 truncation (:146), v_med3_i32
        short o;
        if constexpr (LT::WB) {
            // DC word (bit 30): the value itself -- one sign-extended bit field and one bit-field
            // insert (the compiler's select was and + cmp + cndmask)
            const uint32_t dcm = (uint32_t)__builtin_amdgcn_sbfe((int)w, 30, 1);
            uint32_t ov;
            asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(ov) : "v"(dcm), "v"(w), "v"((uint32_t)v));
            o = (short)ov;
        } else {
            o = (w & MP2VG_COEF_DC) ? (short)level : (short)v;
        }
        // a lane past the group's words writes its (meaningless) value to byte 0 of the wave's
        // residual image instead, which IDCT pass 2 rewrites before the store pass reads it
        if constexpr (LT::WB) {
            // byte address: slot * 128 + ((slot & 7) * 16 XOR doubled scan position)
            const uint32_t a = MP2VG_I_KBTAB
                                   ? (uint32_t)(uintptr_t)(lds_short2_t*)L.blk[wave] + ((kb >> 8) ^ (uint32_t)L.scan[64 * h + i])
                                   : (uint32_t)(uintptr_t)(lds_short2_t*)L.blk[wave] + ((uint32_t)slot << 7) +
                                         ((((uint32_t)slot << 4) & 0x70u) ^ (uint32_t)L.scan[64 * h + i]);
            const uint32_t d = (uint32_t)(uintptr_t)(lds_short2_t*)L.res[wave];
            *(__attribute__((address_space(3))) short*)(uintptr_t)(live ? a : d) = o;
        } else {
            short* const dst = live ? &((short*)L.blk[wave])[LT::bofs(slot, L.scan[64 * h + i])] : (short*)L.res[wave];
            *dst = o;
        }
        return;
    }
    // the word's MB in its group: slices are whole MB rows (plan_batch), so groups start at a
    // column multiple of 4 and the MB is (column mod 8) & 3 = bits 26-27, next to the block
    // (bits 22-25): bits 22-27 index the group's dequant table.  A word's block is coded in its
    // MB's cbp, and DC / '1s' words carry i = 0 (mp2vg_batch_upload rejects batches where not).
    const uint32_t e = L.dq[wave][(w >> 22) & 63u];
    const int slot = (int)(e & 0xff);
    const bool intra = INTRA_ONLY || ((e >> 18) & 1);
    const int qs = (int)((e >> 8) & 0xff);
    const int i = (w >> 16) & 63;
    const int level = (short)(w & 0xffff);
    const bool dc = w & MP2VG_COEF_DC;  // QFS[0] = dc << (3 - prec), outside the parity sum (:160)
    const bool s1 = !INTRA_ONLY && (w & MP2VG_COEF_FIRST1S);
    const int Wi = L.W[4 * h + ((e >> 16) & 3)][i];
    const int sign = level < 0 ? -1 : 0;
    const int mag = level < 0 ? -level : level;
    // W*qs < 2^16 and 2*|level|+1 <= 65537 < 2^24: 24-bit multiplies (full rate) give the low 32
    // bits of the product, i.e. the reference's int arithmetic, where v_mul_lo_u32 is quarter rate
    const uint32_t wq = __umul24((uint32_t)Wi, (uint32_t)qs);
    int val = intra ? (int)mul24_asm((uint32_t)mag, wq) >> 4 : (int)mul24_asm((uint32_t)(2 * mag + 1), wq) >> 5;
    val = (val ^ sign) - sign;
    const int t = (short)val;  // int16 truncation before the clamp (:146)
    short v = (short)min(max(t, -2048), 2047);  // v_med3_i32
    if (!INTRA_ONLY) {  // '1s' first coefficient: (3*W*qs)>>5 at qfs[0], unclamped (:79-88)
        const short t1 = (short)((int)(3u * wq) >> 5);
        v = s1 ? (short)((t1 ^ sign) - sign) : v;
    }
    v = dc ? (short)level : v;  // branch-free: every lane of the word round writes once
    ((short*)L.blk[wave * LT::NBUF + buf])[LT::bofs(slot, L.scan[64 * h + i])] = v;  // i = 0 for DC and '1s' words: block position 0
}

// force the wait for every tap load here (an empty asm reading the registers): a direction
// that no lane uses is skipped by predict(), and a still-pending load would otherwise make the
// compiler wait on it later, behind the stores, when the register is reused
template <int NW>
__device__ __forceinline__ void touch(const Tap<NW>& t) {
#pragma unroll
    for (int i = 0; i <= NW; i++) asm volatile("" ::"v"(t.a[i]), "v"(t.b[i]));
}

// Diagnostic stamp build only (ABL & 16, never in tests or the bench): per-stage s_memtime
// cycle sums per wave, added to a u64 array in the pool's pad (geo.sink + 1024, 8 per mode).
struct Stamps {
    uint64_t t, acc[7];
};
template <int ABL>
__device__ __forceinline__ void stamp(Stamps& st, int i) {
    if (!(ABL & 16)) return;
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    // (the comment names the stage in the assembly: tools/stage_mix.py splits the loop there)
    asm volatile("s_memtime %0 ; stage stamp %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "i"(i) : "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (i >= 0) st.acc[i] += t - st.t;
    st.t = t;
}

// the first 64*NCW coefficient words of a group, one per lane per register: P/B groups carry
// few words (plain loads, the array is padded by 256 words); I groups up to NCW*64 through the
// batch's coefficient buffer resource, registers wholly past the group's words out of range
template <int MCM, int NCW>
__device__ __forceinline__ void prefetch_words(uint32_t (&cw)[NCW], const SliceCtx& c, uint32_t coef0, int ncoef,
                                               int lane) {
    if (MCM != 0) {
#pragma unroll
        for (int j = 0; j < NCW; j++) cw[j] = ld_rec(&c.coefs[coef0 + 64 * j + lane]);
    } else {
        const uint32_t off = (coef0 + (uint32_t)lane) * 4u;
#pragma unroll
        for (int j = 0; j < NCW; j++)
            cw[j] = __builtin_amdgcn_raw_buffer_load_b32(c.coef_rsrc, 64 * j < ncoef ? (int)(off + 256u * j) : (int)kNoTap,
                                                         0, MP2VG_REC_NT ? 2 : 0);
    }
}

// Software pipeline per wave, one iteration per group g (the wave's groups are STEP MBs apart):
//   top:       taps of g have landed (one vmcnt wait) -> prediction P(g) in VGPRs
//   look-ahead: taps of g+1 (records of g+1 arrived one iteration ago), records of g+2
//   C:         dequant of g; then the coefficient words of g+1 (128; I kernels up to 1,536)
//   D, E:      IDCT, add/clip + store of g
// Every look-ahead value is consumed before its register is reloaded (no loop-carried copies of
// pending loads), so the waits at the top never cover the previous group's stores.
template <int CF, int MCM, int ABL, class LT, bool TILES = true>  // TILES: the anchor-tile store code
__device__ __forceinline__ void run_slice(const SliceCtx& c, const Geo& geo, LT& L, int lane, int wave) {
    using F = Fmt<CF>;
    using RL = ResLayout<CF>;
    constexpr int NB = F::NB;
    const uint32_t STEP = c.step;
    constexpr int NWC = F::CW / 4;
    // 4:2:0 intra groups (24 blocks) run both IDCT passes in shared rounds (D' below)
    constexpr bool UNI = LT::COMPACT && CF == 1;
    const uint32_t mb_end = c.mb_end, mb_last = c.mb_end - 1;
    uint32_t g = c.mb_begin + c.wpos * G;
    if (g >= mb_end) return;
    const int kl = lane & 3;

    Tap<4> t0f, t0b;    // luma rows
    Tap<NWC> t1f, t1b;  // chroma rows (4:2:0: Cb + Cr; else Cb)
    Tap<NWC> t2f, t2b;  // Cr rows (4:2:2 / 4:4:4)
    Group S;
    // coefficient words prefetched one group ahead, 64 per register; a word past the prefetch is a
    // synchronous load (a full memory latency).  I pictures (MCM 0) prefetch as many words as a
    // dense intra group carries (4:4:4, 20-40 AC per block: ~1,500; 2,048 measured no faster)
    // with range-checked buffer loads: registers past the group's words load nothing (kNoTap)
    constexpr int NCW = MCM == 0 ? (CF == 3 ? 24 : (CF == 2 ? 12 : 8)) : 2;
    uint32_t gr0, gr1, rvN, cw[NCW];
    bool glive;
    {
        const uint32_t rv = rec_load(c.mbrec, g, mb_last, lane);
        const int ng = (int)min(mb_end - g, (uint32_t)G);
        glive = kl < ng;
        const LaneRec R = lane_rec(rv, lane);
        if (MCM) issue_pass<CF, MCM, 0, 4, ABL>(R, glive, lane, geo, c.ref_fwd, c.ref_bwd, t0f, t0b, c.dir);
        S = group_state<NB>(rv, ng);
        gr0 = R.r0;
        gr1 = R.r1;
        __builtin_amdgcn_sched_barrier(0);
        rvN = rec_load(c.mbrec, g + STEP < mb_end ? g + STEP : g, mb_last, lane);
        prefetch_words<MCM, NCW>(cw, c, S.coef0, S.ncoef, lane);
        __builtin_amdgcn_sched_barrier(0);
        if (MCM) {
            issue_pass<CF, MCM, 1, NWC, ABL>(R, glive, lane, geo, c.cref_fwd, c.cref_bwd, t1f, t1b, c.dir);
            if (CF != 1) issue_pass<CF, MCM, 2, NWC, ABL>(R, glive, lane, geo, c.cref_fwd, c.cref_bwd, t2f, t2b, c.dir);
        }
        __builtin_amdgcn_sched_barrier(0);
        // the steady-state loop issues the group's stores after these loads: dummy stores to the
        // sink give the prologue the same VMEM sequence, so the compiler's merged in-order
        // vmcnt state at the loop head does not degrade to vmcnt(0)
        if (!(ABL & 8)) {
#pragma unroll
            for (int j = 0; j < Passes<CF>::N; j++) ((uint32_t*)c.wsink)[j * 4] = 0u;  // 16 B apart: not merged
        }
    }

    Stamps st;
#pragma unroll
    for (int i = 0; i < 7; i++) st.acc[i] = 0;
    stamp<ABL>(st, -1);
    for (; g < mb_end; g += STEP) {
        stamp<ABL>(st, 6);  // loop overhead (latch)
        // ---- prediction of g from the taps issued one iteration ago ----
        uint32_t p0[4] = {0, 0, 0, 0}, p1[NWC], p2[NWC];
#pragma unroll
        for (int d = 0; d < NWC; d++) p1[d] = p2[d] = 0;
        if (MCM) {
            touch(t0f), touch(t1f);
            if (MCM == 2) touch(t0b), touch(t1b);
            if (CF != 1) touch(t2f);
            if (CF != 1 && MCM == 2) touch(t2b);
            predict<MCM, 4, ABL>(t0f, t0b, lane, p0);
            predict<MCM, NWC, ABL>(t1f, t1b, lane, p1);
            if (CF != 1) predict<MCM, NWC, ABL>(t2f, t2b, lane, p2);
        }

        stamp<ABL>(st, 0);
        // ---- look-ahead: taps of g+1, records of g+2 (group indices clamped in-slice) ----
        const uint32_t gn = g + STEP < mb_end ? g + STEP : g;
        const int ngN = (int)min(mb_end - gn, (uint32_t)G);
        const bool gliveN = kl < ngN;
        const LaneRec R = lane_rec(rvN, lane);
        if (MCM) issue_pass<CF, MCM, 0, 4, ABL>(R, gliveN, lane, geo, c.ref_fwd, c.ref_bwd, t0f, t0b, c.dir);
        const Group SN = group_state<NB>(rvN, ngN);
        __builtin_amdgcn_sched_barrier(0);
        rvN = rec_load(c.mbrec, g + 2 * STEP < mb_end ? g + 2 * STEP : g, mb_last, lane);

        stamp<ABL>(st, 1);
        // ---- C. slot map + dequant (parse_block, mb_decoder.cpp:74-155) ----
        if constexpr (MCM != 0) {  // I pictures need neither (dequant_word / slot_kb)
            const uint32_t e = dq_entry<CF>(S, lane);
            L.dq[wave][lane] = e;
            if (e & (1u << 19)) L.map[wave][e & 0xff] = (uint8_t)lane;
            wave_sync();
        }
        if (!(ABL & 4)) {
            // words 0..64*NCW-1 from the registers loaded one group ahead; more (rare) loaded here
            if constexpr (MCM == 0) {
                // I pictures: registers up to the group's last word, lanes past it masked by their
                // store address rather than by exec (no divergent branch per word register)
#pragma unroll
                for (int j = 0; j < NCW; j++) {
                    if (64 * j >= S.ncoef) break;
                    dequant_word<LT, true, NB>(L, wave, cw[j], S.qs8, 64 * j + lane < S.ncoef, c.half);
                }
            } else {
#pragma unroll
                for (int j = 0; j < NCW; j++)
                    if (64 * j + lane < S.ncoef) dequant_word<LT, false, NB>(L, wave, cw[j], S.qs8, true, c.half);
            }
            // words past the prefetch: XW loads per lane in flight per round trip, not one (a 4:4:4
            // intra group carries ~1,400 words)
            constexpr int XW = MCM == 0 ? 8 : 2;
            if (S.ncoef > 64 * NCW) {
                for (int base = 64 * NCW; base < S.ncoef; base += 64 * XW) {
                    uint32_t xw[XW];
#pragma unroll
                    for (int j = 0; j < XW; j++) {
                        const int wi = base + 64 * j + lane;
                        xw[j] = wi < S.ncoef ? ld_rec(&c.coefs[S.coef0 + wi]) : 0u;
                    }
#pragma unroll
                    for (int j = 0; j < XW; j++)
                        if (base + 64 * j + lane < S.ncoef) dequant_word<LT, MCM == 0, NB>(L, wave, xw[j], S.qs8, true, c.half);
                }
                // Drain this rare path's loads before it rejoins: the waitcnt pass merges the
                // paths' pending-load state, and a load it cannot prove retired (a lane-masked
                // one) made it put a vmcnt(0) -- every tap of g+1 and the previous stores in
                // flight -- on the common path, once per group.
                __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
            }
        }
        // first 64*NCW coefficient words of g+1 (the words of g are consumed)
        __builtin_amdgcn_sched_barrier(0);
        prefetch_words<MCM, NCW>(cw, c, SN.coef0, SN.ncoef, lane);
        __builtin_amdgcn_sched_barrier(0);
        wave_sync();

        stamp<ABL>(st, 2);
        // dev ablations (timing only): IDCT pass 2 (131072) or both passes (262144) skipped in
        // every second group of the wave -- the bound of pooling two groups' IDCT rounds
        bool odd = false;
        if constexpr ((ABL & (131072 | 262144)) != 0) odd = ((g - c.mb_begin) / STEP) & 1;
        if constexpr (!UNI) {
            // ---- D. IDCT pass 1 (idct_sse2.hpp:102-103): lane (slot, v, v+1) transforms coefficient
            //         rows v, v+1 over u.  Mismatch control (mb_decoder.cpp:150-152; intra DC
            //         excluded, :76) is folded in: the block parity is reduced over the slot's 4
            //         lanes with ds_swizzle and applied to QFS[63] (row 7, u 7) before the
            //         transform.  Output transposed in place ([x][v]): the block is read by one
            //         ds_read instruction before any lane writes it.
            for (int t = lane; t < (((ABL & 1) || ((ABL & 262144) && odd)) ? 0 : S.nslots * 4); t += 64) {
                const int slot = t >> 2, v = (t & 3) * 2;
                short* const bw = (short*)L.blk[wave];
                lds_uint4_t *pa, *pb;
                slot_chunks<LT>(bw, slot, v, v + 1, pa, pb);
                uint4 ra = ld16(pa);
                uint4 rb = ld16(pb);
                const int k = slot_kb<MCM, NB>(L, wave, slot) >> 4;
                const bool intra = MCM == 0 || (pick8(S.fl8, k) & MP2VG_MB_INTRA);
                uint32_t par = (ra.x ^ ra.y ^ ra.z ^ ra.w ^ rb.x ^ rb.y ^ rb.z ^ rb.w) & 0x00010001u;
                if (v == 0 && intra) par ^= ra.x & 1u;  // DC excluded
                par = (par ^ (par >> 16)) & 1u;
                par ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)par, 0x041F);  // xor lane 1
                par ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)par, 0x081F);  // xor lane 2
                if (v == 6) rb.w ^= (par ^ 1u) << 16;  // sum even -> toggle the LSB of QFS[63]
                // pair-interleaved block: dword u = (row v, row v + 1) of column u, no unpacking
                short2_t s[8] = {__builtin_bit_cast(short2_t, ra.x), __builtin_bit_cast(short2_t, ra.y),
                                 __builtin_bit_cast(short2_t, ra.z), __builtin_bit_cast(short2_t, ra.w),
                                 __builtin_bit_cast(short2_t, rb.x), __builtin_bit_cast(short2_t, rb.y),
                                 __builtin_bit_cast(short2_t, rb.z), __builtin_bit_cast(short2_t, rb.w)};
                idct_1d<true>(s);
                pass1_store<LT>(bw, slot, v, s);
            }
            wave_sync();
            // chroma taps of g+1 issued mid-iteration: spreads the wave's TA demand
            __builtin_amdgcn_sched_barrier(0);
            if (MCM) {
                issue_pass<CF, MCM, 1, NWC, ABL>(R, gliveN, lane, geo, c.cref_fwd, c.cref_bwd, t1f, t1b, c.dir);
                if (CF != 1) issue_pass<CF, MCM, 2, NWC, ABL>(R, gliveN, lane, geo, c.cref_fwd, c.cref_bwd, t2f, t2b, c.dir);
            }
            __builtin_amdgcn_sched_barrier(0);
            stamp<ABL>(st, 3);
            // pass 2 (:104-108): lane (slot, x, x+2) transforms columns x, x+2 over v; >>6 -> residual
            // image in the MB's dct_type placement (:166-196); the block area is zeroed for the next
            // group
            for (int t = lane; t < (((ABL & 1) || ((ABL & (131072 | 262144)) && odd)) ? 0 : S.nslots * 4); t += 64) {
                const int slot = t >> 2, xq = t & 3;
                const int x = (xq & 1) | ((xq & 2) << 1);  // 0, 1, 4, 5
                short* const bw = (short*)L.blk[wave];
                lds_uint4_t *pa, *pb;
                slot_chunks<LT>(bw, slot, x, x + 2, pa, pb);
                const uint4 ra = ld16(pa);
                const uint4 rb = ld16(pb);
                zero16(pa);
                zero16(pb);
                short2_t s[8];
                interleave(ra, rb, s);
                idct_1d(s);
                const int kb = slot_kb<MCM, NB>(L, wave, slot);
                const int k = kb >> 4, bb = kb & 15;
                const bool dctf = pick8(S.fl8, k) & MP2VG_MB_DCT_FIELD;
                int plane, x0, y0, ys;
                block_origin<CF>(bb, dctf, plane, x0, y0, ys);
                const int rw = RL::width(plane);
                const int xp = RL::pos(x0 + x);  // (x, x+2) -> (xp, xp+1)
                if constexpr (LT::COMPACT) {
                    // intra put (idct_sse2.hpp:106-108): packus(res) -- the clamped bytes of (x, x+2)
                    const uint32_t a0 = (uint32_t)(uintptr_t)(lds_u16_t*)((uint8_t*)L.res[wave] + RL::base(plane)) +
                                        mul24_asm((uint32_t)k, (uint32_t)RL::SIZE) + (uint32_t)(y0 * rw + xp);
                    put8_rows(a0, (uint32_t)(ys * rw), s);
                } else {
                    // row y at a0 + y * step, one add per row (see put8_rows)
                    const uint32_t a0 = (uint32_t)(uintptr_t)(lds_short2_t*)(&L.res[wave][RL::base(plane)]) +
                                        2u * (mul24_asm((uint32_t)k, (uint32_t)RL::MBS) + (uint32_t)(y0 * rw + xp));
                    const uint32_t step = 2u * (uint32_t)(ys * rw);
#pragma unroll
                    for (int y = 0; y < 8; y++) *(lds_short2_t*)(uintptr_t)(a0 + (uint32_t)y * step) = s[y] >> (short)6;
                }
            }
            wave_sync();
        } else {
            // ---- D'. 4:2:0 intra: both IDCT passes in shared rounds.  A group's 24 blocks are 96
            //          pass-1 items and 96 pass-2 items; item slots 0..95 are pass 1, 96..191 pass
            //          2, three rounds of 64 instead of two half-empty rounds per pass.  A pass-2
            //          item always lands in a later round than its block's pass-1 items (it sits
            //          >= 64 slots after them), so one wave_sync per round orders them; within a
            //          round the two passes touch different blocks.  The per-item work is the
            //          pass-1 / pass-2 code below, unchanged.
            const int n4 = S.nslots * 4;
            const int p2b = n4 > 64 ? n4 : 64;
            short* const bw = (short*)L.blk[wave];
            for (int base = 0; base < ((ABL & 1) ? 0 : p2b + n4); base += 64) {
                const int t = base + lane;
                const bool p1 = t < n4;
                const int u = p1 ? t : t - p2b;
                if (p1 || (t >= p2b && u < n4)) {
                    const int slot = u >> 2, q = u & 3;
                    const int v = q * 2;                           // pass 1: rows v, v+1
                    const int x = (q & 1) | ((q & 2) << 1);       // pass 2: columns x, x+2 (0, 1, 4, 5)
                    // the item's two 16-B chunks (pass 1: rows v, v+1; pass 2: columns x, x+2); pass 2
                    // zeroes them after reading
                    lds_uint4_t *pa, *pb;
                    slot_chunks<LT>(bw, slot, p1 ? v : x, p1 ? v + 1 : x + 2, pa, pb);
                    uint4 ra = ld16(pa);
                    uint4 rb = ld16(pb);
                    short2_t sv[8];
                    if (p1) {
                        // mismatch control (intra: DC excluded), as in pass 1 above
                        uint32_t par = (ra.x ^ ra.y ^ ra.z ^ ra.w ^ rb.x ^ rb.y ^ rb.z ^ rb.w) & 0x00010001u;
                        if (v == 0) par ^= ra.x & 1u;
                        par = (par ^ (par >> 16)) & 1u;
                        par ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)par, 0x041F);
                        par ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)par, 0x081F);
                        if (v == 6) rb.w ^= (par ^ 1u) << 16;
                        sv[0] = __builtin_bit_cast(short2_t, ra.x), sv[1] = __builtin_bit_cast(short2_t, ra.y);
                        sv[2] = __builtin_bit_cast(short2_t, ra.z), sv[3] = __builtin_bit_cast(short2_t, ra.w);
                        sv[4] = __builtin_bit_cast(short2_t, rb.x), sv[5] = __builtin_bit_cast(short2_t, rb.y);
                        sv[6] = __builtin_bit_cast(short2_t, rb.z), sv[7] = __builtin_bit_cast(short2_t, rb.w);
                    } else {
                        zero16(pa);
                        zero16(pb);
                        interleave(ra, rb, sv);
                    }
                    if (base + 64 <= n4)
                        idct_1d<true>(sv);
                    else
                        idct_1d(sv);
                    if (p1) {
                        pass1_store<LT>(bw, slot, v, sv);
                    } else {
                        const int kb = slot_kb<MCM, NB>(L, wave, slot);
                        const int k = kb >> 4, bb = kb & 15;
                        const bool dctf = pick8(S.fl8, k) & MP2VG_MB_DCT_FIELD;
                        int plane, x0, y0, ys;
                        block_origin<CF>(bb, dctf, plane, x0, y0, ys);
                        const int rw = RL::width(plane);
                        const int xp = RL::pos(x0 + x);
                        const uint32_t a0 = (uint32_t)(uintptr_t)(lds_u16_t*)((uint8_t*)L.res[wave] + RL::base(plane)) +
                                            mul24_asm((uint32_t)k, (uint32_t)RL::SIZE) + (uint32_t)(y0 * rw + xp);
                        put8_rows(a0, (uint32_t)(ys * rw), sv);
                    }
                }
                wave_sync();
            }
            stamp<ABL>(st, 3);
        }

        stamp<ABL>(st, 4);
        // ---- E. prediction + residual, one row store per lane ----
        if constexpr (LT::COMPACT) {
            const uint8_t* res8 = (const uint8_t*)L.res[wave];
            store_pass_put8<CF, 0, 4>(gr0, glive, lane, geo, c.wsink, c.dst_slot, c.dst_rsrc, res8);
            store_pass_put8<CF, 1, NWC>(gr0, glive, lane, geo, c.wsink, c.dst_slot, c.dst_rsrc, res8);
            if (CF != 1) store_pass_put8<CF, 2, NWC>(gr0, glive, lane, geo, c.wsink, c.dst_slot, c.dst_rsrc, res8);
            if (TILES && c.tiles) {  // MB 0 of the group is always live
                const uint32_t r00 = (uint32_t)__builtin_amdgcn_readfirstlane((int)gr0);
                tile_group<CF, false, ABL>(r00 & 0xffff, r00 >> 16, lane, geo, c.wsink, c.dst_tiles, c.tile_rsrc, res8);
            }
        } else {
            store_pass<CF, 0, 4, ABL>(gr0, gr1, glive, lane, geo, c.wsink, c.dst_slot, c.dst_rsrc, MCM != 2 && c.tiles, L.res[wave], p0);
            store_pass<CF, 1, NWC, ABL>(gr0, gr1, glive, lane, geo, c.wsink, c.dst_slot, c.dst_rsrc, MCM != 2 && c.tiles, L.res[wave], p1);
            if (CF != 1) store_pass<CF, 2, NWC, ABL>(gr0, gr1, glive, lane, geo, c.wsink, c.dst_slot, c.dst_rsrc, MCM != 2 && c.tiles, L.res[wave], p2);
            if (MCM != 2 && c.tiles) {  // the pixels store_pass left in the residual image, as whole tile lines
                wave_sync();
                const uint32_t r00 = (uint32_t)__builtin_amdgcn_readfirstlane((int)gr0);
                tile_group<CF, true, ABL>(r00 & 0xffff, r00 >> 16, lane, geo, c.wsink, c.dst_tiles, c.tile_rsrc,
                                          (const uint8_t*)L.res[wave]);
            }
        }
        wave_sync();

        stamp<ABL>(st, 5);
        S = SN;
        gr0 = R.r0;
        gr1 = R.r1;
        glive = gliveN;
    }
    if ((ABL & 16) && lane == 0) {
        unsigned long long* out = (unsigned long long*)(geo.sink + 1024) + 8 * MCM;
#pragma unroll
        for (int i = 0; i < 7; i++) atomicAdd(&out[i], (unsigned long long)st.acc[i]);
        atomicAdd(&out[7], 1ull);
    }
}

// Occupancy targets per kernel from its LDS: 4:2:0 / 4:2:2 P/B workgroups fit 4 per CU (128
// VGPRs), 4:4:4 P/B 3 (168 VGPRs cost nothing); the compact I kernels fit 4 (4:4:4) or 6 (80 VGPRs)
template <int CF, int MCM, int ABL = 0>
// MCM: 0 I pictures, 1 P, 2 B, 3 a mixed P/B level (the picture type picks the loop per
// workgroup), 4 I pictures without the anchor-tile store code (I-only launches where few pictures
// store tiles: theirs are converted after the launch, runtime.cpp TilePlan)
__global__ __launch_bounds__((64 * kernel_waves<MCM, ABL>())) __attribute__((amdgpu_waves_per_eu((MCM == 0 || MCM == 4) && (ABL & ~kAblCompact) == 0 ? (CF == 3 ? 4 : 6) : (CF == 3 ? 3 : 4)))) void recon_kernel(const mp2vg_picture_t* __restrict__ pics,
                                                    const uint32_t* __restrict__ mbrec,
                                                    const uint32_t* __restrict__ coefs,
                                                    const SliceDesc* __restrict__ slices,
                                                    const Geo geo,
                                                    const uint32_t slice_base, const uint32_t nslices,
                                                    const uint32_t mates) {
    using LT = Lds<CF, compact_layout<MCM, ABL>(), kernel_waves<MCM, ABL>()>;
    __shared__ __attribute__((aligned(128))) LT L;  // 128-B aligned: pass1_store
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // Work units: one slice, or with `mates` (P/B launches, runtime.cpp plan_batch) two
    // consecutive slices -- cluster mates, the same MB row of two pictures that read the same
    // references -- waves 0-1 on the first, 2-3 on the second.  XCD-aware bijection: XCD x = b % 8
    // owns the contiguous unit range [x*q + min(x, r), ...)
    static_assert(slices_per_wg<CF, MCM, ABL>(4) <= (uint32_t)LT::NH, "one matrix set per slice");
    const uint32_t spw = slices_per_wg<CF, MCM, ABL>(mates);  // the grid's rule (launch_one)
    const bool two = spw > 1;
    const uint32_t wps = 4u / spw;  // waves per slice
    const uint32_t nunits = (nslices + spw - 1) / spw;
    const uint32_t b = blockIdx.x, q8 = nunits / 8, r8 = nunits % 8, xcd = b % 8;
    const uint32_t unit = xcd * q8 + min(xcd, r8) + b / 8;
    const int half = two ? (int)((uint32_t)wave / wps) : 0;
    const uint32_t si = spw * unit + (uint32_t)half;
    const bool have = si < nslices;  // (the last unit may hold fewer slices)
    const SliceDesc sd = slices[slice_base + min(si, nslices - 1)];  // in range for every wave
    const mp2vg_picture_t* pic = pics + sd.pic;
    const int alt = pic->alternate_scan & 1;

    if ((uint32_t)wave % wps == 0 && (two || tid < 64)) {
        ((uint32_t*)L.W)[64 * half + lane] = ((const uint32_t*)pic->W)[lane];
        // blocks sit in LDS pair-interleaved: coefficient (v, u) at (v >> 1) * 16 + u * 2 + (v & 1),
        // so a dword is the (row v, row v + 1) pair of column u that IDCT pass 1 transforms
        const int r = c_scan_raster[alt][lane];
        const int pos = (r >> 4) * 16 + (r & 7) * 2 + ((r >> 3) & 1);
        L.scan[64 * half + lane] = (uint8_t)(LT::WB ? 2 * pos : pos);
        if constexpr (LT::WB && MP2VG_I_KBTAB) {
            const int k = lane >> 4, bb = lane & 15;
            const uint32_t slot = (uint32_t)(k * Fmt<CF>::NB + (bb < Fmt<CF>::NB ? bb : 0));
            L.kbtab[lane] = (((slot << 7) | ((slot << 4) & 0x70u)) << 8) | ((uint32_t)k * 8u);
        }
        if constexpr (LT::WB && CF != 1) {
#pragma unroll
            for (int bb = 0; bb < Fmt<CF>::NB; bb++) L.Wb[bb][lane] = pic->W[bb < 6 ? 0 : 2][lane];
        }
    }
    for (int i = lane; i < LT::NBUF * LT::MAXS * LT::BLK / 2; i += 64) ((uint32_t*)L.blk[wave * LT::NBUF])[i] = 0;
    __syncthreads();
    if (!have) return;

    SliceCtx c;
    c.mbrec = mbrec;
    c.coefs = coefs;
    c.dst_slot = (uint8_t*)geo.ftab[pic->dst_slot];
    c.wsink = geo.sink + 2048 + ((b * LT::NWAVES + wave) & 1023) * 64;
    c.dst_tiles = (uint8_t*)geo.ttab[pic->dst_slot];
    c.dst_rsrc = slot_rsrc(c.dst_slot, (uint32_t)geo.slot_bytes);
    c.tile_rsrc = slot_rsrc(c.dst_tiles, (uint32_t)(2 * geo.slot_bytes));
    c.tiles = sd.reserved & 1u;
    // SliceDesc.reserved bit 1: a B picture that predicts in one direction only, run by the
    // one-reference loop (MCM 1); bit 2: that direction is backward (runtime.cpp plan_batch)
    const bool one_dir = sd.reserved & 2u;
    c.dir = (sd.reserved >> 2) & 1u;
    // the taps read the references' anchor tiles (tile slot = 2 x slot bytes)
    const int fs0 = pic->fwd_slot < 0 ? pic->dst_slot : pic->fwd_slot;
    const int bs = pic->bwd_slot < 0 ? pic->dst_slot : pic->bwd_slot;
    const int fs = c.dir ? bs : fs0;
    c.ref_fwd = slot_rsrc((const uint8_t*)geo.ttab[fs], (uint32_t)(2 * geo.slot_bytes));
    c.ref_bwd = slot_rsrc((const uint8_t*)geo.ttab[bs], (uint32_t)(2 * geo.slot_bytes));
    if (kChromaTiles) {
        c.cref_fwd = c.ref_fwd, c.cref_bwd = c.ref_bwd;
    } else {
        c.cref_fwd = slot_rsrc((const uint8_t*)geo.ftab[fs], (uint32_t)geo.slot_bytes);
        c.cref_bwd = slot_rsrc((const uint8_t*)geo.ftab[bs], (uint32_t)geo.slot_bytes);
    }
    c.coef_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)coefs, (short)0, (int)kNoTap, 0x00020000);
    c.mb_begin = sd.mb_begin;
    c.mb_end = sd.mb_begin + sd.mb_count;
    c.half = half;
    c.wpos = two ? (uint32_t)wave % wps : (uint32_t)wave;
    c.step = (two ? wps : (uint32_t)LT::NWAVES) * G;
    if constexpr (MCM == 4) {
        run_slice<CF, 0, ABL, LT, false>(c, geo, L, lane, wave);
    } else if constexpr (MCM < 3) {
        run_slice<CF, (ABL & 2) ? 0 : MCM, ABL, LT>(c, geo, L, lane, wave);
    } else {  // mixed level: the picture type picks the specialised loop (uniform per workgroup)
        const int pct = pic->picture_coding_type;
        if (pct == 3 && !one_dir)
            run_slice<CF, (ABL & 2) ? 0 : 2, ABL, LT>(c, geo, L, lane, wave);
        else if (pct == 2 || one_dir)
            run_slice<CF, (ABL & 2) ? 0 : 1, ABL, LT>(c, geo, L, lane, wave);
        else
            run_slice<CF, 0, ABL, LT>(c, geo, L, lane, wave);
    }
}
// Order-independent 64-bit digest of a slot's visible planes:
//   sum over visible dwords d at (row_id, byte x) of mix64(mix64((row_id << 32) | x) ^ d)   (mod 2^64)
// (rows numbered across Y, U, V).  The outer mix makes each term a pseudo-random function of the
// dword, so sparse +-1 errors cannot cancel pairwise in the sum (an additive key ^ d term could).  tiny_mp2v_dec_amd.records.planes_digest is the host twin.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void digest_kernel(const uint64_t* __restrict__ ftab, const int32_t* __restrict__ slots,
                              uint64_t o0, uint64_t o1, uint64_t o2, int s0, int s1, int w0, int w1, int h0, int h1,
                              unsigned long long* __restrict__ out) {
    const int si = blockIdx.y;
    const uint8_t* base = (const uint8_t*)ftab[slots[si]];
    const int rows = h0 + 2 * h1;
    uint64_t acc = 0;
    for (int row = blockIdx.x; row < rows; row += gridDim.x) {
        const uint8_t* p;
        int w;
        if (row < h0) {
            p = base + o0 + (uint64_t)row * s0;
            w = w0;
        } else if (row < h0 + h1) {
            p = base + o1 + (uint64_t)(row - h0) * s1;
            w = w1;
        } else {
            p = base + o2 + (uint64_t)(row - h0 - h1) * s1;
            w = w1;
        }
        for (int x = threadIdx.x * 4; x < w; x += blockDim.x * 4) {
            const uint32_t d = *(const uint32_t*)(p + x);
            acc += mix64(mix64(((uint64_t)row << 32) | (uint64_t)x) ^ (uint64_t)d);
        }
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0) atomicAdd(&out[si], (unsigned long long)acc);
}

template <int CF, int MCM, int ABL>
static void launch_one(const KArgs& a, const Geo& g, hipStream_t stream) {
    const uint32_t spw = slices_per_wg<CF, MCM, ABL>(a.mates);  // the kernel applies the same rule
    hipLaunchKernelGGL((recon_kernel<CF, MCM, ABL>), dim3((a.nslices + spw - 1) / spw),
                       dim3(64 * kernel_waves<MCM, ABL>()), 0, stream, a.pics, (const uint32_t*)a.mbs, a.coefs,
                       a.slices, g, a.slice_base, a.nslices, spw);
}

template <int CF, int ABL>
static hipError_t launch_mcm(int mcm, const KArgs& a, const Geo& g, hipStream_t stream) {
    switch (mcm) {
    case 0: launch_one<CF, 0, ABL>(a, g, stream); break;
    case 1: launch_one<CF, 1, ABL>(a, g, stream); break;
    case 2: launch_one<CF, 2, ABL>(a, g, stream); break;
    case 3: launch_one<CF, 3, ABL>(a, g, stream); break;
    case 4: launch_one<CF, 4, ABL>(a, g, stream); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_recon(int cf, int mcm, const KArgs& a, hipStream_t stream) {
    Geo g;
    g.sink = a.sink;
    g.slot_bytes = a.slot_bytes;
    g.ftab = a.ftab;
    g.ttab = a.ttab;
    for (int i = 0; i < 3; i++) {
        g.plane_off[i] = (uint32_t)a.plane_off[i];
        g.stride[i] = a.stride[i];
        g.ph[i] = a.ph[i];
    }
    // development-only ablation switch (MP2VG_ABLATE; compiled only into dev builds with
    // -DMP2VG_DEV_ABLATIONS, tools/variant.sh EXTRA=...; 4:2:0, and 16 also 4:4:4): 1 no IDCT, 2 no
    // MC, 4 no dequant, 8 no stores, 16 stage stamps (tools/stamps.py), 32 MC loads out of range
    // (no address math), 64 no prediction arithmetic, 128 no 17th-pixel dwords, 512 no edge-row
    // loads, 2048 all-hit taps, 4096/8192 store shapes, 32768 none.  Outputs are wrong under
    // it (except 16); never set in tests or the bench.  A product library refuses the variable.
    static const int ablate = getenv("MP2VG_ABLATE") ? atoi(getenv("MP2VG_ABLATE")) : 0;
#ifndef MP2VG_DEV_ABLATIONS
    if (ablate) return hipErrorNotSupported;
#else
    if (cf == 3 && ablate == 16) return launch_mcm<3, 16>(mcm, a, g, stream);
    if (cf == 1 && ablate) {
        switch (ablate) {
        case 1: return launch_mcm<1, 1>(mcm, a, g, stream);
        case 2: return launch_mcm<1, 2>(mcm, a, g, stream);
        case 4: return launch_mcm<1, 4>(mcm, a, g, stream);
        case 8: return launch_mcm<1, 8>(mcm, a, g, stream);
        case 15: return launch_mcm<1, 15>(mcm, a, g, stream);
        case 16: return launch_mcm<1, 16>(mcm, a, g, stream);
        case 32: return launch_mcm<1, 32>(mcm, a, g, stream);
        case 64: return launch_mcm<1, 64>(mcm, a, g, stream);
        case 96: return launch_mcm<1, 96>(mcm, a, g, stream);
        case 128: return launch_mcm<1, 128>(mcm, a, g, stream);
        case 512: return launch_mcm<1, 512>(mcm, a, g, stream);
        case 2048: return launch_mcm<1, 2048>(mcm, a, g, stream);
        case 2056: return launch_mcm<1, 2056>(mcm, a, g, stream);
        case 4096: return launch_mcm<1, 4096>(mcm, a, g, stream);
        case 8192: return launch_mcm<1, 8192>(mcm, a, g, stream);
        case 32768: return launch_mcm<1, 32768>(mcm, a, g, stream);  // no-op: the dev build's own baseline
        case 65536: return launch_mcm<1, 65536>(mcm, a, g, stream);  // tile stores in a 64-KB window
        case 131072: return launch_mcm<1, 131072>(mcm, a, g, stream);  // pass 2 in every 2nd group only
        case 262144: return launch_mcm<1, 262144>(mcm, a, g, stream);  // IDCT in every 2nd group only
        default: return hipErrorInvalidValue;
        }
    }
#endif
    switch (cf) {
    case 1: return launch_mcm<1, 0>(mcm, a, g, stream);
    case 2: return launch_mcm<2, 0>(mcm, a, g, stream);
    case 3: return launch_mcm<3, 0>(mcm, a, g, stream);
    default: return hipErrorInvalidValue;
    }
}

// Slots' anchor tiles built from their frames, in whole 128-B lines (runtime.cpp TilePlan: the B
// pictures of a launch that later pictures read, right after it, and any reference whose writer
// stored none).  A tile row is the frame row's bytes [W t, W t + 2 W): thread = one 16-B
// chunk of a tile line (8 per line), read straight from the frame row.  Picture = blockIdx.y:
// slot list[y] (or slot0 without a list).
__global__ void __launch_bounds__(256) tile_convert_kernel(const Geo geo, int cw, const int32_t* __restrict__ list,
                                                           int32_t slot0) {
    const int32_t slot = list ? list[blockIdx.y] : slot0;
    const uint8_t* frame = (const uint8_t*)geo.ftab[slot];
    uint8_t* tiles = (uint8_t*)geo.ttab[slot];
#pragma unroll
    for (int plane = 0; plane < 3; plane++) {
        const int w = plane == 0 ? 16 : cw;       // tile width class
        const int R = w == 16 ? 4 : 8, RB = 128 / R;  // rows per tile, bytes per tile row
        const uint32_t ncol = (uint32_t)geo.stride[plane] / w;
        const uint32_t n = (uint32_t)geo.ph[plane] / R * ncol * 8;  // 16-B chunks of the plane
        for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
            const uint32_t line = i >> 3, c = i & 7;
            const uint32_t band = line / ncol, t = line % ncol;
            const uint32_t r = c / (RB / 16), o = (c % (RB / 16)) * 16;
            const uint8_t* src = frame + geo.plane_off[plane] + (size_t)(band * R + r) * geo.stride[plane] + t * w + o;
            const uint2 lo = *(const uint2*)src, hi = *(const uint2*)(src + 8);
            *(uint4*)(tiles + 2 * (size_t)geo.plane_off[plane] + (size_t)line * 128 + c * 16) =
                make_uint4(lo.x, lo.y, hi.x, hi.y);
        }
    }
}

hipError_t launch_tile_convert(const KArgs& a, int cf, const int32_t* d_list, int n, int32_t slot0, hipStream_t stream) {
    Geo g;
    g.ftab = a.ftab;
    g.ttab = a.ttab;
    for (int i = 0; i < 3; i++) {
        g.plane_off[i] = (uint32_t)a.plane_off[i];
        g.stride[i] = a.stride[i];
        g.ph[i] = a.ph[i];
    }
    const int cw = cf == 3 ? 16 : 8;  // chroma MB width
    hipLaunchKernelGGL(tile_convert_kernel, dim3(128, d_list ? n : 1), dim3(256), 0, stream, g, cw, d_list, slot0);
    return hipGetLastError();
}

// Decoded slots -> the drop-in's pinned host frames (decoder.cpp), one launch per chunk: the copy
// kernel's stores go straight over PCIe into host memory.  Measured on the box (tools/
// d2h_kernel_probe.hip, 1080p 4:2:0 frames): 54 GB/s for 16 frames over 64 workgroups against
// 47.5 GB/s for one hipMemcpyAsync (SDMA) per frame, and it leaves the DMA engines to the uploads.
// Blocks (x, f) stride over frame f's 16-B units; a tail of bytes % 16 goes byte by byte.
__global__ void __launch_bounds__(256) frame_copy_kernel(FrameCopy fc, uint64_t bytes) {
    typedef uint32_t u4v_t __attribute__((ext_vector_type(4)));
    const int f = blockIdx.y;
    const uint8_t* __restrict__ src = fc.src[f];
    uint8_t* __restrict__ dst = fc.dst[f];
    const uint64_t n16 = bytes >> 4, step = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += step)
        ((u4v_t*)dst)[i] = ((const u4v_t*)src)[i];
    if (blockIdx.x == 0)
        for (uint64_t i = (n16 << 4) + threadIdx.x; i < bytes; i += 256) dst[i] = src[i];
}

hipError_t launch_frame_copy(const FrameCopy& fc, int n, uint64_t bytes, hipStream_t stream) {
    if (n < 1 || n > kFrameCopyMax) return hipErrorInvalidValue;
    for (int i = 0; i < n; i++)
        if (((uintptr_t)fc.src[i] | (uintptr_t)fc.dst[i]) & 15) return hipErrorInvalidValue;
    // about 64 workgroups per launch: PCIe-bound, so few waves; the rest of the chip stays with
    // the next chunk's decode
    static const int wgs = getenv("MP2VG_DL_WGS") ? std::max(1, atoi(getenv("MP2VG_DL_WGS"))) : 64;  // (measurements)
    dim3 block(256), grid(n < wgs ? wgs / n : 1, n);
    hipLaunchKernelGGL(frame_copy_kernel, grid, block, 0, stream, fc, bytes);
    return hipGetLastError();
}

// Shader clock under a VALU load on every SIMD (bench.py's per-box record): each wave runs a chain
// of dependent-free v_add/v_xor for `iters` iterations between two s_memtime / s_memrealtime
// pairs (s_memtime counts shader cycles, s_memrealtime a constant 100 MHz); out[0] += cycles,
// out[1] += 100-MHz ticks, summed over waves.  Read-only timers, vector stores only.
__global__ void __launch_bounds__(256) clock_probe_kernel(unsigned long long* __restrict__ out, int iters) {
    uint32_t a = threadIdx.x, b = a * 2654435761u, c2 = a ^ 0x9e3779b9u, d = ~a;
    uint64_t t0, r0, t1, r1;
    asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0)::"memory");
    for (int i = 0; i < iters; i++) {
        asm volatile("v_add_u32 %0, %0, %1\n v_xor_b32 %1, %1, %2\n v_add_u32 %2, %2, %3\n v_xor_b32 %3, %3, %0"
                     : "+v"(a), "+v"(b), "+v"(c2), "+v"(d));
    }
    asm volatile("s_memtime %0\n s_memrealtime %1\n s_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1)::"memory");
    if ((a ^ b ^ c2 ^ d) == 0x12345678u) out[2] = 1;  // keeps the chain live
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&out[0], (unsigned long long)(t1 - t0));
        atomicAdd(&out[1], (unsigned long long)(r1 - r0));
    }
}

hipError_t launch_clock_probe(unsigned long long* d_out, int iters, int blocks, hipStream_t stream) {
    hipLaunchKernelGGL(clock_probe_kernel, dim3(blocks), dim3(256), 0, stream, d_out, iters);
    return hipGetLastError();
}

// Pool-placement probe over one pool block, contents kept: every 16-B word is loaded and (rw)
// stored back xor `zero` (a runtime 0, so the store is not folded away).  Read-only sweeps fold the
// words into one store per lane to the sink only when the fold equals `zero`'s complement.
template <bool RW>
__global__ void __launch_bounds__(256) block_probe_kernel(u4v* __restrict__ p, size_t n, uint32_t zero, int reps,
                                                          u4v* __restrict__ sink) {
    u4v acc = {0, 0, 0, 0};
    for (int r = 0; r < reps; r++)
        for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
            u4v v = p[i];
            if (RW) {
                v.x ^= zero;
                p[i] = v;
            } else {
                acc ^= v;
            }
        }
    if (!RW && (acc.x ^ acc.y ^ acc.z ^ acc.w) == ~zero) sink[threadIdx.x] = acc;
}

// Pool-placement probe over the whole pool: every wave reads `iters` 1-KB runs (16 B per lane).
// LOCK = false: each run in a random slot (frame or tile), at a random 1-KB offset (a page-walk /
// TLB-reach probe); true: wave w reads slot w % nslots, and run i of every wave sits at the same
// offset i * 4 KB in its slot (many pictures at one offset at once: the decode's access shape).
template <bool LOCK, bool RW = false>
__global__ void __launch_bounds__(256) pool_scatter_kernel(const uint64_t* __restrict__ tab, int nslots,
                                                           uint32_t fkb, uint32_t tkb, int iters,
                                                           u4v* __restrict__ sink, uint32_t zero) {
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    u4v acc = {0, 0, 0, 0};
    uint32_t h = wave * 2654435761u + 12345u;
    for (int i = 0; i < iters; i++) {
        uint32_t slot, tile, kb;
        if (LOCK) {
            slot = wave % nslots;
            tile = wave / nslots & 1;
            kb = (uint32_t)i * 4 % (tile ? tkb : fkb);
        } else {
            h ^= h << 13, h ^= h >> 17, h ^= h << 5;
            slot = h % nslots;
            tile = h >> 31;
            const uint32_t g = h * 0x9e3779b1u;
            kb = (g >> 8) % (tile ? tkb : fkb);
        }
        u4v* p = (u4v*)(tab[tile * nslots + slot] + (uint64_t)kb * 1024) + lane;
        u4v v = *p;
        if (RW) {  // stored back unchanged (xor a runtime 0)
            v.x ^= zero;
            *p = v;
        } else {
            acc ^= v;
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == ~zero) sink[threadIdx.x] = acc;
}

// Random 1-KB reads inside one pool block (its pages only): a block mapped in small fragments
// needs more translation entries than the per-CU / per-XCD TLBs hold.
__global__ void __launch_bounds__(256) block_random_kernel(const uint8_t* __restrict__ base, uint32_t kbs, int iters,
                                                           u4v* __restrict__ sink, uint32_t zero) {
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    u4v acc = {0, 0, 0, 0};
    uint32_t h = wave * 2654435761u + 777u;
    for (int i = 0; i < iters; i++) {
        h ^= h << 13, h ^= h >> 17, h ^= h << 5;
        const uint32_t kb = (h * 0x9e3779b1u >> 8) % kbs;
        acc ^= *((const u4v*)(base + (uint64_t)kb * 1024) + lane);
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == ~zero) sink[threadIdx.x] = acc;
}

hipError_t launch_block_random(const void* base, size_t bytes, int waves, int iters, void* sink, hipStream_t stream) {
    hipLaunchKernelGGL(block_random_kernel, dim3(waves / 4), dim3(256), 0, stream, (const uint8_t*)base,
                       (uint32_t)(bytes >> 10), iters, (u4v*)sink, 0u);
    return hipGetLastError();
}

hipError_t launch_pool_scatter(const uint64_t* tab, int nslots, uint32_t fkb, uint32_t tkb, int lock, int waves,
                               int iters, void* sink, hipStream_t stream) {
    if (lock >= 2)  // 2: same offsets, loaded and stored back; 3: random, loaded and stored back
        hipLaunchKernelGGL((lock == 2 ? pool_scatter_kernel<true, true> : pool_scatter_kernel<false, true>),
                           dim3(waves / 4), dim3(256), 0, stream, tab, nslots, fkb, tkb, iters, (u4v*)sink, 0u);
    else if (lock)
        hipLaunchKernelGGL(pool_scatter_kernel<true>, dim3(waves / 4), dim3(256), 0, stream, tab, nslots, fkb, tkb,
                           iters, (u4v*)sink, 0u);
    else
        hipLaunchKernelGGL(pool_scatter_kernel<false>, dim3(waves / 4), dim3(256), 0, stream, tab, nslots, fkb, tkb,
                           iters, (u4v*)sink, 0u);
    return hipGetLastError();
}

hipError_t launch_block_probe(void* p, size_t bytes, int rw, int reps, void* sink, hipStream_t stream) {
    const size_t n = bytes / 16;
    if (rw)
        hipLaunchKernelGGL(block_probe_kernel<true>, dim3(2048), dim3(256), 0, stream, (u4v*)p, n, 0u, reps, (u4v*)sink);
    else
        hipLaunchKernelGGL(block_probe_kernel<false>, dim3(2048), dim3(256), 0, stream, (u4v*)p, n, 0u, reps, (u4v*)sink);
    return hipGetLastError();
}

hipError_t launch_digest(const uint64_t* ftab, const int32_t* d_slots, int n,
                         const uint64_t off[3], const int32_t stride[3], const int32_t w[3],
                         const int32_t h[3], unsigned long long* d_out, hipStream_t stream) {
    dim3 block(256), grid(64, n);
    hipLaunchKernelGGL(digest_kernel, grid, block, 0, stream, ftab, d_slots, off[0], off[1], off[2],
                       stride[0], stride[1], w[0], w[1], h[0], h[1], d_out);
    return hipGetLastError();
}

}  // namespace mp2vg
