// recon.hip — HIP kernels of the macroblock reconstruct path (gfx950 / CDNA4 only: wave64,
// packed 16-bit VALU, v_lerp_u8, LDS per wave; no CUDA-compat layer).  See recon_kernel.h for
// the map to the reference.
//
// Work decomposition: one workgroup (4 waves) per slice (= MB row, XCD-aware order); each wave
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
__device__ __forceinline__ short2_t mulhi2(short2_t a, int c) {
    short2_t r;
    r.x = (short)(((int)a.x * c) >> 16);
    r.y = (short)(((int)a.y * c) >> 16);
    return r;
}

// idct_sse2.hpp:23-65, two lanes of the SSE2 vector at once
__device__ __forceinline__ void idct_1d(short2_t s[8]) {
    const short2_t v15 = adds2(shl2(mulhi2(s[0], 27145), 1), shl2(s[0], 1));
    const short2_t v26 = adds2(mulhi2(s[1], -5037), shl2(s[1], 2));
    const short2_t v21 = adds2(mulhi2(s[2], -19954), shl2(s[2], 2));
    const short2_t v28 = adds2(shl2(mulhi2(s[3], -22089), 1), shl2(s[3], 2));
    const short2_t v16 = adds2(shl2(mulhi2(s[4], 27145), 1), shl2(s[4], 1));
    const short2_t v25 = adds2(mulhi2(s[5], 14567), shl2(s[5], 1));
    const short2_t v22 = adds2(shl2(mulhi2(s[6], 17391), 1), s[6]);
    const short2_t v27 = shl2(mulhi2(s[7], 25570), 1);
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
    const short2_t v12 = subs2(v18, adds2(v19, mulhi2(v19, 20090)));  // op3
    const short2_t v14 = subs2(subs2(v20, mulhi2(v20, 30068)), v18);  // op1
    const short2_t v6 = subs2(shl2(v14, 1), v7);
    const short2_t v5 = subs2(adds2(v13, mulhi2(v13, 27145)), v6);    // op0
    const short2_t v4 = adds2(v5, shl2(v12, 1));
    const short2_t v10 = subs2(adds2(v17, mulhi2(v17, 27145)), v11);  // op0
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

// per-byte (a + b + 1) >> 1 on 4 packed u8 == _mm_avg_epu8: one v_lerp_u8 (rounding bit per byte)
__device__ __forceinline__ uint32_t avg4(uint32_t a, uint32_t b) { return __builtin_amdgcn_lerp(a, b, 0x01010101u); }

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
constexpr int G = 4;  // macroblocks per wave group

// Residual image of one MB in LDS (int16): luma 16x16, then Cb CW x CH, then Cr.  Inside each
// group of 4 pixels the order is x0, x0+2, x0+1, x0+3: one v_perm unpacks the matching
// prediction bytes into (x0, x0+2) / (x0+1, x0+3) pairs for packed i16 math, and IDCT pass 2
// (columns x, x+2 per lane) stores one dword per output row.
template <int CF>
struct ResLayout {
    using F = Fmt<CF>;
    static constexpr int SIZE = 256 + 2 * F::CW * F::CH;
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

// Per-MB wave-uniform state of a group (SGPRs).  Fields are 4-vectors with named components:
// with plain arrays the compiler lowers the per-lane pick() below into a lane-indexed SCRATCH
// load of a stack copy of the group.
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
struct Group {
    u4v mbx, mby, flags, cbp, qs, mv[4];  // mv[r*2+s], component k = MB
    u4v slot_base, coef_rel;
    int nslots, ncoef;
    uint32_t coef0;
};

// select component k (lane-varying) of a wave-uniform 4-vector: three v_cndmask
__device__ __forceinline__ uint32_t pick(const u4v& v, int k) {
    return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w));
}

// Pixel-row passes of a group: pass 0 = the 64 luma rows (4 MBs x 16); 4:2:0 pass 1 = Cb + Cr
// (4 x 8 each); 4:2:2 / 4:4:4 pass 1 = Cb, pass 2 = Cr (4 x 16 each).  Rows of the same pixel
// row of adjacent MBs sit in adjacent lanes.
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

// one prediction direction of one pixel row: raw dwords from the dword-aligned reference x
template <int NW>  // output dwords: 4 (16-px row) or 2 (8-px row)
struct RowTap {
    static constexpr int ND = NW + 1;  // dwords loaded per reference row
    uint32_t a[ND], b[ND];             // rows Y and Y + step
    int sh, hxy;
};

template <int CF, int NW>
__device__ __forceinline__ void row_tap_issue(RowTap<NW>& t, const uint8_t* __restrict__ plane_base, uint32_t mvw,
                                              int plane, int gx, int py, int mby_base, bool field, int fs, int stride,
                                              int ph) {
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
    } else {  // field MC (mb_decoder.cpp:229-236): rows 2q + field_select, vector r = py & 1
        Y = mby_base + fs + 2 * ((py >> 1) + (mvy >> 1));
        step = 2;
    }
    // clamp into the plane so out-of-contract vectors can never fault (inactive in contract)
    const int Xc = min(max(X, 0), stride - 4);
    const int Y0 = min(max(Y, 0), ph - 1);
    const int Y1 = min(max(Y + step, 0), ph - 1);
    t.sh = Xc & 3;
    t.hxy = (mvx & 1) | ((mvy & 1) << 1);
    const uint32_t* r0 = (const uint32_t*)(plane_base + (size_t)Y0 * stride + (Xc & ~3));
#pragma unroll
    for (int i = 0; i < RowTap<NW>::ND; i++) t.a[i] = r0[i];
    if (t.hxy & 2) {
        const uint32_t* r1 = (const uint32_t*)(plane_base + (size_t)Y1 * stride + (Xc & ~3));
#pragma unroll
        for (int i = 0; i < RowTap<NW>::ND; i++) t.b[i] = r1[i];
    } else {
#pragma unroll
        for (int i = 0; i < RowTap<NW>::ND; i++) t.b[i] = t.a[i];
    }
}

// cascaded half-pel average of one row (mc_sse2.hpp:5-39 == mc_c.hpp:15), branch-free:
// avg(x, x) == x, so the unused taps are replaced by the used ones.
template <int NW>
__device__ __forceinline__ void row_tap_finish(const RowTap<NW>& t, uint32_t (&p)[4]) {
    const uint32_t s = (uint32_t)t.sh;
    const bool hx = t.hxy & 1;
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
        const uint32_t B = __builtin_amdgcn_alignbyte(A[d + 1], A[d], 1u);
        const uint32_t D = __builtin_amdgcn_alignbyte(C[d + 1], C[d], 1u);
        const uint32_t r0 = avg4(A[d], hx ? B : A[d]);
        const uint32_t r1 = avg4(C[d], hx ? D : C[d]);
        p[d] = avg4(r0, r1);  // r1 == r0 when the vector is vertically full-pel
    }
}

template <int CF, int ABL>
struct Kern {
    using F = Fmt<CF>;
    using RL = ResLayout<CF>;
    static constexpr int NB = F::NB;
    static constexpr int MAXS = G * NB;  // coded-block slots per group
    static constexpr int NWC = F::CW / 4;  // dwords per chroma row
};

template <int CF, int J, int NW>
__device__ __forceinline__ void issue_pass(const Group& S, int lane, const Geo& geo, const uint8_t* ref_fwd,
                                           const uint8_t* ref_bwd, RowTap<NW>& tf, RowTap<NW>& tb, bool skip) {
    using F = Fmt<CF>;
    int k, plane, py;
    pass_row<CF, J>(lane, k, plane, py);
    const uint32_t fl = pick(S.flags, k);
    const bool none = (fl & MP2VG_MB_INTRA) || skip;
    const bool bwd = fl & MP2VG_MB_BWD;
    const bool fwd = !none && ((fl & MP2VG_MB_FWD) || !bwd);
    const bool field = fl & MP2VG_MB_FIELD_MC;
    const int pw = plane == 0 ? 16 : F::CW;
    const int phm = plane == 0 ? 16 : F::CH;
    const int gx = (int)pick(S.mbx, k) * pw;
    const int mbyb = (int)pick(S.mby, k) * phm;
    const int r = field ? (py & 1) : 0;
    const int stride = gsel(geo.stride, plane);
    const int ph = gsel(geo.ph, plane);
    tf.hxy = tb.hxy = 0;
    tf.sh = tb.sh = 0;
    if (fwd) {
        const uint32_t mvw = r ? pick(S.mv[2], k) : pick(S.mv[0], k);
        row_tap_issue<CF, NW>(tf, ref_fwd + gsel(geo.plane_off, plane), mvw, plane, gx, py, mbyb, field,
                              (fl >> (8 + 2 * r)) & 1, stride, ph);
    }
    if (!none && bwd) {
        const uint32_t mvw = r ? pick(S.mv[3], k) : pick(S.mv[1], k);
        row_tap_issue<CF, NW>(tb, ref_bwd + gsel(geo.plane_off, plane), mvw, plane, gx, py, mbyb, field,
                              (fl >> (9 + 2 * r)) & 1, stride, ph);
    }
}

template <int CF, int J, int NW, int ABL>
__device__ __forceinline__ void finish_pass(const Group& S, int ng, int lane, const Geo& geo, uint8_t* dst_slot,
                                            const short* s_res_wave, const RowTap<NW>& tf, const RowTap<NW>& tb) {
    using F = Fmt<CF>;
    using RL = ResLayout<CF>;
    int k, plane, py;
    pass_row<CF, J>(lane, k, plane, py);
    if (k >= ng) return;
    const uint32_t fl = pick(S.flags, k);
    const bool intra = fl & MP2VG_MB_INTRA;
    const bool bwd = fl & MP2VG_MB_BWD;
    const bool fwd = !intra && ((fl & MP2VG_MB_FWD) || !bwd);
    uint32_t p[4] = {0, 0, 0, 0};
    if (!intra) {
        uint32_t pf[4] = {0, 0, 0, 0}, pb[4] = {0, 0, 0, 0};
        if (fwd) row_tap_finish<NW>(tf, pf);
        if (bwd) row_tap_finish<NW>(tb, pb);
#pragma unroll
        for (int d = 0; d < NW; d++) p[d] = (fwd && bwd) ? avg4(pf[d], pb[d]) : (fwd ? pf[d] : pb[d]);  // mc_sse2.hpp:78-84
    }
    // put: packus(res); add: packus(adds(pred, res))   (idct_sse2.hpp:106-119)
    const uint32_t cbpk = pick(S.cbp, k);
    const int lb = left_block<CF>(plane, py, fl & MP2VG_MB_DCT_FIELD);
    const int rb = (plane == 0) ? lb + 1 : lb + 4;
    const bool cl = cbpk & (1u << lb);
    const bool cr = NW == 4 && (cbpk & (1u << rb));
    uint32_t out[4] = {p[0], p[1], p[2], p[3]};
    if (cl || cr) {
        const short* res = s_res_wave + k * RL::SIZE + RL::base(plane) + py * RL::width(plane);
        uint32_t rv[8];
        const uint4 r0 = *(const uint4*)&res[0];
        rv[0] = r0.x; rv[1] = r0.y; rv[2] = r0.z; rv[3] = r0.w;
        if (NW == 4) {
            const uint4 r1 = *(const uint4*)&res[8];
            rv[4] = r1.x; rv[5] = r1.y; rv[6] = r1.z; rv[7] = r1.w;
        }
#pragma unroll
        for (int d = 0; d < NW; d++) {
            if (!(d < 2 ? cl : cr)) continue;
            // pairs (x0, x0+2) and (x0+1, x0+3) as packed i16
            const uint32_t lo = __builtin_amdgcn_perm(0u, p[d], 0x0c020c00u);
            const uint32_t hi = __builtin_amdgcn_perm(0u, p[d], 0x0c030c01u);
            short2_t a = __builtin_bit_cast(short2_t, lo) + __builtin_bit_cast(short2_t, rv[2 * d]);
            short2_t c = __builtin_bit_cast(short2_t, hi) + __builtin_bit_cast(short2_t, rv[2 * d + 1]);
            const short2_t z = {0, 0}, m = {255, 255};
            a = __builtin_elementwise_min(__builtin_elementwise_max(a, z), m);
            c = __builtin_elementwise_min(__builtin_elementwise_max(c, z), m);
            // bytes: x0 = a.lo, x0+1 = c.lo, x0+2 = a.hi, x0+3 = c.hi
            out[d] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, c), __builtin_bit_cast(uint32_t, a), 0x06020400u);
        }
    }
    const int pw = plane == 0 ? 16 : F::CW;
    const int phm = plane == 0 ? 16 : F::CH;
    uint8_t* dst = dst_slot + gsel(geo.plane_off, plane) +
                   (size_t)((int)pick(S.mby, k) * phm + py) * gsel(geo.stride, plane) + (int)pick(S.mbx, k) * pw;
    if (ABL & 8) {
        asm volatile("" ::"v"(out[0]), "v"(out[1]), "v"(out[2]), "v"(out[3]));
    } else if (NW == 4) {
        *(uint4*)dst = make_uint4(out[0], out[1], out[2], out[3]);
    } else {
        *(uint2*)dst = make_uint2(out[0], out[1]);
    }
}

template <int CF, int ABL = 0>
__global__ __launch_bounds__(256) void recon_kernel(const mp2vg_picture_t* __restrict__ pics,
                                                    const uint32_t* __restrict__ mbrec,
                                                    const uint32_t* __restrict__ coefs,
                                                    const SliceDesc* __restrict__ slices,
                                                    uint8_t* __restrict__ pool, const Geo geo,
                                                    const uint32_t slice_base, const uint32_t nslices) {
    using F = Fmt<CF>;
    using RL = ResLayout<CF>;
    constexpr int NB = F::NB;
    constexpr int MAXS = G * NB;
    constexpr int NWC = F::CW / 4;
    __shared__ __attribute__((aligned(16))) short s_blk[WAVES][MAXS][64];  // coef raster -> pass-1 out
    __shared__ __attribute__((aligned(16))) short s_res[WAVES][G * RL::SIZE];
    __shared__ uint8_t s_map[WAVES][MAXS];  // slot -> k*16 + b
    __shared__ uint8_t s_W[4][64];
    __shared__ uint8_t s_scan[64];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // XCD-aware bijection: XCD x = b % 8 owns the contiguous slice range [x*q + min(x, r), ...)
    const uint32_t b = blockIdx.x, q8 = nslices / 8, r8 = nslices % 8, xcd = b % 8;
    const uint32_t si = xcd * q8 + min(xcd, r8) + b / 8;
    const SliceDesc sd = slices[slice_base + si];
    const mp2vg_picture_t* pic = pics + sd.pic;
    const int alt = pic->alternate_scan & 1;

    if (tid < 64) {
        ((uint32_t*)s_W)[tid] = ((const uint32_t*)pic->W)[tid];
        s_scan[tid] = c_scan_raster[alt][tid];
    }
    for (int i = lane; i < MAXS * 64 / 2; i += 64) ((uint32_t*)s_blk[wave])[i] = 0;
    __syncthreads();

    uint8_t* const dst_slot = pool + (uint64_t)pic->dst_slot * geo.slot_bytes;
    const uint8_t* const ref_fwd = pool + (uint64_t)(pic->fwd_slot < 0 ? pic->dst_slot : pic->fwd_slot) * geo.slot_bytes;
    const uint8_t* const ref_bwd = pool + (uint64_t)(pic->bwd_slot < 0 ? pic->dst_slot : pic->bwd_slot) * geo.slot_bytes;

    const uint32_t mb_end = sd.mb_begin + sd.mb_count;
    for (uint32_t g0 = sd.mb_begin + wave * G; g0 < mb_end; g0 += WAVES * G) {
        // ---- A. group records: uniform scalar loads (the MB array is padded by 16 records);
        //         readfirstlane pins them in SGPRs (else the compiler turns the per-lane pick<>
        //         selects back into lane-indexed vector loads of the record) ----
        const int ng = min((int)(mb_end - g0), G);
        Group S;
        int sb = 0, cr = 0;
        const uint32_t* rp = mbrec + (size_t)g0 * 8;
#define SLD(i) ((uint32_t)__builtin_amdgcn_readfirstlane((int)rp[i]))
        S.coef0 = SLD(3);
#pragma unroll
        for (int k = 0; k < G; k++) {
            const uint32_t r0 = SLD(k * 8 + 0), r1 = SLD(k * 8 + 1), r2 = SLD(k * 8 + 2);
            const bool live = k < ng;
            const uint32_t cbpk = live ? ((r1 >> 16) & ((1u << NB) - 1)) : 0u;
            S.mbx[k] = r0 & 0xffff;
            S.mby[k] = r0 >> 16;
            S.flags[k] = live ? (r1 & 0xffff) : (uint32_t)MP2VG_MB_INTRA;
            S.cbp[k] = cbpk;
            S.qs[k] = r2 & 0xff;
            S.slot_base[k] = (uint32_t)sb;
            S.coef_rel[k] = (uint32_t)cr;
            sb += __builtin_popcount(cbpk);
            cr += live ? (int)(r2 >> 16) : 0;
#pragma unroll
            for (int q = 0; q < 4; q++) S.mv[q][k] = SLD(k * 8 + 4 + q);
        }
#undef SLD
        S.nslots = sb;
        S.ncoef = cr;
        const uint32_t cw0 = lane < S.ncoef ? coefs[S.coef0 + lane] : 0u;

        // ---- B. reference-row loads of every pixel row (consumed in E) ----
        RowTap<4> t0f, t0b;   // luma rows
        RowTap<NWC> t1f, t1b;  // chroma rows (4:2:0: Cb + Cr; else Cb)
        RowTap<NWC> t2f, t2b;  // Cr rows (4:2:2 / 4:4:4)
        issue_pass<CF, 0, 4>(S, lane, geo, ref_fwd, ref_bwd, t0f, t0b, ABL & 2);
        issue_pass<CF, 1, NWC>(S, lane, geo, ref_fwd, ref_bwd, t1f, t1b, ABL & 2);
        if (CF != 1) issue_pass<CF, 2, NWC>(S, lane, geo, ref_fwd, ref_bwd, t2f, t2b, ABL & 2);

        // ---- C. slot map + dequant (parse_block, mb_decoder.cpp:74-155) ----
        if (lane < MAXS) {
            const int k = lane / NB, bb = lane % NB;
            const uint32_t cbpk = pick(S.cbp, k);
            if (cbpk & (1u << bb))
                s_map[wave][(int)pick(S.slot_base, k) + __builtin_popcount(cbpk & ((1u << bb) - 1))] = (uint8_t)(k * 16 + bb);
        }
        for (int k0 = 0; k0 < ((ABL & 4) ? 0 : S.ncoef); k0 += 64) {
            const int w_idx = k0 + lane;
            const uint32_t w = k0 == 0 ? cw0 : (w_idx < S.ncoef ? coefs[S.coef0 + w_idx] : 0u);
            if (w_idx >= S.ncoef) continue;
            int k = 0;
#pragma unroll
            for (int i = 1; i < G; i++) k += (w_idx >= (int)S.coef_rel[i]) ? 1 : 0;
            const uint32_t cbpk = pick(S.cbp, k);
            const int bb = (w >> 22) & 15;
            if (bb >= NB || !(cbpk & (1u << bb))) continue;  // host validation rejects these
            const int slot = (int)pick(S.slot_base, k) + __builtin_popcount(cbpk & ((1u << bb) - 1));
            const bool intra = pick(S.flags, k) & MP2VG_MB_INTRA;
            const int qs = (int)pick(S.qs, k);
            const int i = (w >> 16) & 63;
            const int level = (short)(w & 0xffff);
            if (w & MP2VG_COEF_DC) {  // QFS[0] = dc << (3 - prec), outside the parity sum (:160)
                s_blk[wave][slot][0] = (short)level;
                continue;
            }
            const int Wi = s_W[(bb < 6 ? 0 : 2) + (intra ? 0 : 1)][i];
            const int sign = level < 0 ? -1 : 0;
            const int mag = level < 0 ? -level : level;
            short v;
            int pos;
            if (w & MP2VG_COEF_FIRST1S) {  // (3*W*qs)>>5 at qfs[0], unclamped (:79-88)
                const short t = (short)((3 * Wi * qs) >> 5);
                v = (short)((t ^ sign) - sign);
                pos = 0;
            } else {
                int val = intra ? (mag * Wi * qs) >> 4 : ((2 * mag + 1) * Wi * qs) >> 5;
                val = (val ^ sign) - sign;
                const short t = (short)val;  // int16 truncation before the clamp (:146)
                v = t > 2047 ? (short)2047 : (t < -2048 ? (short)-2048 : t);
                pos = s_scan[i];
            }
            s_blk[wave][slot][pos] = v;
        }
        wave_sync();

        // ---- D. IDCT pass 1 (idct_sse2.hpp:102-103): lane (slot, v, v+1) transforms coefficient
        //         rows v, v+1 over u.  Mismatch control (mb_decoder.cpp:150-152; intra DC
        //         excluded, :76) is folded in: the block parity is reduced over the slot's 4
        //         lanes with ds_swizzle and applied to QFS[63] (row 7, u 7) before the
        //         transform.  Output transposed in place ([x][v]): the block is read by one
        //         ds_read instruction before any lane writes it.
        for (int t = lane; t < ((ABL & 1) ? 0 : S.nslots * 4); t += 64) {
            const int slot = t >> 2, v = (t & 3) * 2;
            uint4 ra = *(const uint4*)&s_blk[wave][slot][v * 8];
            uint4 rb = *(const uint4*)&s_blk[wave][slot][v * 8 + 8];
            const int k = s_map[wave][slot] >> 4;
            const bool intra = pick(S.flags, k) & MP2VG_MB_INTRA;
            uint32_t par = (ra.x ^ ra.y ^ ra.z ^ ra.w ^ rb.x ^ rb.y ^ rb.z ^ rb.w) & 0x00010001u;
            if (v == 0 && intra) par ^= ra.x & 1u;  // DC excluded
            par = (par ^ (par >> 16)) & 1u;
            par ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)par, 0x041F);  // xor lane 1
            par ^= (uint32_t)__builtin_amdgcn_ds_swizzle((int)par, 0x081F);  // xor lane 2
            if (v == 6) rb.w ^= (par ^ 1u) << 16;  // sum even -> toggle the LSB of QFS[63]
            short2_t s[8];
            interleave(ra, rb, s);
            idct_1d(s);
#pragma unroll
            for (int x = 0; x < 8; x++) *(short2_t*)&s_blk[wave][slot][x * 8 + v] = s[x];
        }
        wave_sync();
        // pass 2 (:104-108): lane (slot, x, x+2) transforms columns x, x+2 over v; >>6 -> residual
        // image in the MB's dct_type placement (:166-196); the block area is zeroed for the next
        // group
        for (int t = lane; t < ((ABL & 1) ? 0 : S.nslots * 4); t += 64) {
            const int slot = t >> 2, xq = t & 3;
            const int x = (xq & 1) | ((xq & 2) << 1);  // 0, 1, 4, 5
            const uint4 ra = *(const uint4*)&s_blk[wave][slot][x * 8];
            const uint4 rb = *(const uint4*)&s_blk[wave][slot][x * 8 + 16];
            *(uint4*)&s_blk[wave][slot][x * 8] = make_uint4(0, 0, 0, 0);
            *(uint4*)&s_blk[wave][slot][x * 8 + 16] = make_uint4(0, 0, 0, 0);
            short2_t s[8];
            interleave(ra, rb, s);
            idct_1d(s);
            const int kb = s_map[wave][slot];
            const int k = kb >> 4, bb = kb & 15;
            const bool dctf = pick(S.flags, k) & MP2VG_MB_DCT_FIELD;
            int plane, x0, y0, ys;
            block_origin<CF>(bb, dctf, plane, x0, y0, ys);
            short* res = &s_res[wave][k * RL::SIZE + RL::base(plane)];
            const int rw = RL::width(plane);
            const int xp = RL::pos(x0 + x);  // (x, x+2) -> (xp, xp+1)
#pragma unroll
            for (int y = 0; y < 8; y++) *(short2_t*)&res[(y0 + y * ys) * rw + xp] = s[y] >> (short)6;
        }
        wave_sync();

        // ---- E. prediction + residual, one row store per lane ----
        finish_pass<CF, 0, 4, ABL>(S, ng, lane, geo, dst_slot, s_res[wave], t0f, t0b);
        finish_pass<CF, 1, NWC, ABL>(S, ng, lane, geo, dst_slot, s_res[wave], t1f, t1b);
        if (CF != 1) finish_pass<CF, 2, NWC, ABL>(S, ng, lane, geo, dst_slot, s_res[wave], t2f, t2b);
        wave_sync();
    }
}

// Order-independent 64-bit digest of a slot's visible planes:
//   sum over visible dwords d at (row_id, byte x) of mix64((row_id << 32) | x) ^ d   (mod 2^64)
// (rows numbered across Y, U, V).  tiny_mp2v_dec_amd.records.planes_digest is the host twin.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void digest_kernel(const uint8_t* __restrict__ pool, uint64_t slot_bytes, const int32_t* __restrict__ slots,
                              uint64_t o0, uint64_t o1, uint64_t o2, int s0, int s1, int w0, int w1, int h0, int h1,
                              unsigned long long* __restrict__ out) {
    const int si = blockIdx.y;
    const uint8_t* base = pool + (uint64_t)slots[si] * slot_bytes;
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
            acc += mix64(((uint64_t)row << 32) | (uint64_t)x) ^ (uint64_t)d;
        }
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0) atomicAdd(&out[si], (unsigned long long)acc);
}

hipError_t launch_recon(int cf, const KArgs& a, hipStream_t stream) {
    dim3 grid(a.nslices), block(256);
    Geo g;
    g.slot_bytes = a.slot_bytes;
    for (int i = 0; i < 3; i++) {
        g.plane_off[i] = a.plane_off[i];
        g.stride[i] = a.stride[i];
        g.ph[i] = a.ph[i];
    }
    const uint32_t* mb = (const uint32_t*)a.mbs;
    // development-only ablation switch (MP2VG_ABLATE, 4:2:0 only): 1 no IDCT, 2 no MC loads,
    // 4 no dequant, 8 no stores.  Outputs are wrong under it; never set in tests or the bench.
    static const int ablate = getenv("MP2VG_ABLATE") ? atoi(getenv("MP2VG_ABLATE")) : 0;
    if (cf == 1 && ablate) {
#define ABL_CASE(v) \
    case v: hipLaunchKernelGGL((recon_kernel<1, v>), grid, block, 0, stream, a.pics, mb, a.coefs, a.slices, a.pool, g, a.slice_base, a.nslices); break;
        switch (ablate) {
            ABL_CASE(1) ABL_CASE(2) ABL_CASE(3) ABL_CASE(4) ABL_CASE(8) ABL_CASE(15)
        default: return hipErrorInvalidValue;
        }
#undef ABL_CASE
        return hipGetLastError();
    }
    switch (cf) {
    case 1: hipLaunchKernelGGL((recon_kernel<1>), grid, block, 0, stream, a.pics, mb, a.coefs, a.slices, a.pool, g, a.slice_base, a.nslices); break;
    case 2: hipLaunchKernelGGL((recon_kernel<2>), grid, block, 0, stream, a.pics, mb, a.coefs, a.slices, a.pool, g, a.slice_base, a.nslices); break;
    case 3: hipLaunchKernelGGL((recon_kernel<3>), grid, block, 0, stream, a.pics, mb, a.coefs, a.slices, a.pool, g, a.slice_base, a.nslices); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_digest(const uint8_t* pool, uint64_t slot_bytes, const int32_t* d_slots, int n,
                         const uint64_t off[3], const int32_t stride[3], const int32_t w[3],
                         const int32_t h[3], unsigned long long* d_out, hipStream_t stream) {
    dim3 block(256), grid(64, n);
    hipLaunchKernelGGL(digest_kernel, grid, block, 0, stream, pool, slot_bytes, d_slots, off[0], off[1], off[2],
                       stride[0], stride[1], w[0], w[1], h[0], h[1], d_out);
    return hipGetLastError();
}

}  // namespace mp2vg
