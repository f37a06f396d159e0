// recon.hip — HIP kernels of the macroblock reconstruct path (see recon_kernel.h for the map to
// the reference).  Written for gfx950 only: wave64, LDS per wave, no CUDA-compat layer.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "recon_kernel.h"

namespace mp2vg {

// ------------------------------------------------------------------------------------------
// 16-bit saturating helpers (SSE2 semantics: _mm_adds/_mm_subs_epi16 saturate, _mm_slli_epi16
// wraps, _mm_mulhi_epi16 = (a*b)>>16).
__device__ __forceinline__ short adds16(short a, short b) { return __builtin_elementwise_add_sat(a, b); }
__device__ __forceinline__ short subs16(short a, short b) { return __builtin_elementwise_sub_sat(a, b); }
__device__ __forceinline__ short mulhi16(short a, int c) { return (short)(((int)a * c) >> 16); }
__device__ __forceinline__ short shl16(short a, int n) { return (short)((unsigned short)a << n); }

// idct_sse2.hpp:23-65 for one lane
__device__ __forceinline__ void idct_1d(short s[8]) {
    const short v15 = adds16(shl16(mulhi16(s[0], 27145), 1), shl16(s[0], 1));
    const short v26 = adds16(mulhi16(s[1], -5037), shl16(s[1], 2));
    const short v21 = adds16(mulhi16(s[2], -19954), shl16(s[2], 2));
    const short v28 = adds16(shl16(mulhi16(s[3], -22089), 1), shl16(s[3], 2));
    const short v16 = adds16(shl16(mulhi16(s[4], 27145), 1), shl16(s[4], 1));
    const short v25 = adds16(mulhi16(s[5], 14567), shl16(s[5], 1));
    const short v22 = adds16(shl16(mulhi16(s[6], 17391), 1), s[6]);
    const short v27 = shl16(mulhi16(s[7], 25570), 1);
    const short v19 = subs16(v25, v28);
    const short v20 = subs16(v26, v27);
    const short v23 = adds16(v26, v27);
    const short v24 = adds16(v25, v28);
    const short v7 = adds16(v23, v24);
    const short v11 = adds16(v21, v22);
    const short v13 = subs16(v23, v24);
    const short v17 = subs16(v21, v22);
    const short v8 = adds16(v15, v16);
    const short v9 = subs16(v15, v16);
    const short v18 = mulhi16(subs16(v19, v20), 25079);
    const short v12 = subs16(v18, adds16(v19, mulhi16(v19, 20090)));
    const short v14 = subs16(subs16(v20, mulhi16(v20, 30068)), v18);
    const short v6 = subs16(shl16(v14, 1), v7);
    const short v5 = subs16(adds16(v13, mulhi16(v13, 27145)), v6);
    const short v4 = adds16(v5, shl16(v12, 1));
    const short v10 = subs16(adds16(v17, mulhi16(v17, 27145)), v11);
    const short v0 = adds16(v8, v11);
    const short v1 = adds16(v9, v10);
    const short v2 = subs16(v9, v10);
    const short v3 = subs16(v8, v11);
    s[0] = adds16(v0, v7);
    s[1] = adds16(v1, v6);
    s[2] = adds16(v2, v5);
    s[3] = subs16(v3, v4);
    s[4] = adds16(v3, v4);
    s[5] = subs16(v2, v5);
    s[6] = subs16(v1, v6);
    s[7] = subs16(v0, v7);
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

// SWAR per-byte rounding-up average: (a + b + 1) >> 1 on 4 packed u8 (== _mm_avg_epu8)
__device__ __forceinline__ uint32_t avg4(uint32_t a, uint32_t b) {
    return (a | b) - (((a ^ b) >> 1) & 0x7f7f7f7fu);
}

// 5 consecutive bytes at p (any alignment) -> {bytes 0..3, bytes 1..4}
__device__ __forceinline__ void load5(const uint8_t* p, uint32_t& lo, uint32_t& sh1) {
    uintptr_t a = (uintptr_t)p;
    const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
    uint32_t s = (uint32_t)(a & 3) * 8;
    uint64_t v = ((uint64_t)w[1] << 32) | w[0];
    v >>= s;
    lo = (uint32_t)v;
    sh1 = (uint32_t)(v >> 8);
}

template <int CF>
struct Fmt {
    static constexpr int NB = CF == 1 ? 6 : (CF == 2 ? 8 : 12);  // blocks per MB
    static constexpr int CW = CF == 3 ? 16 : 8;                  // chroma MB width
    static constexpr int CH = CF == 1 ? 8 : 16;                  // chroma MB height
    static constexpr int ITEMS = 64 + 2 * (CW / 4) * CH;         // 4-pixel items per MB
};

// which coded block covers MB-plane pixel row py / column px (mb_decoder.cpp:176-195)
template <int CF>
__device__ __forceinline__ int block_of(int plane, int px, int py, bool dctf) {
    if (plane == 0) return (dctf ? (py & 1) : (py >> 3)) * 2 + (px >> 3);
    int base = plane == 1 ? 4 : 5;
    if (CF == 1) return base;
    bool lower = (dctf ? (py & 1) : (py >> 3)) != 0;
    int k = (px >= 8 ? 2 : 0) + (lower ? 1 : 0);
    return base + 2 * k;
}

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
    int k = (b - 4) >> 1;
    x0 = k >= 2 ? 8 : 0;
    bool lower = (k & 1);
    if (dctf && CF != 1) {
        y0 = lower ? 1 : 0;
        ys = 2;
    } else {
        y0 = lower ? 8 : 0;
    }
}

constexpr int WAVES = 4;

// Residual image of one MB in LDS: luma 16x16, then Cb CW x CH, then Cr (int16)
template <int CF>
struct ResLayout {
    using F = Fmt<CF>;
    static constexpr int SIZE = 256 + 2 * F::CW * F::CH;
    __device__ static constexpr int base(int plane) { return plane == 0 ? 0 : 256 + (plane - 1) * F::CW * F::CH; }
    __device__ static constexpr int width(int plane) { return plane == 0 ? 16 : F::CW; }
};

// item index (G MBs side by side) -> MB k, plane, pixel column px (multiple of 4), row py.
// Items of one pixel row of the group are consecutive so a row of lanes stores 16*G contiguous
// bytes of luma (4*CW*G/4 of chroma).
template <int CF, int G>
__device__ __forceinline__ void item_coords(int it, int& k, int& plane, int& px, int& py) {
    using F = Fmt<CF>;
    constexpr int LUMA = G * 64;
    constexpr int CPR = F::CW / 4;       // chroma items per MB row
    constexpr int CPL = G * CPR * F::CH;  // chroma items per plane
    if (it < LUMA) {
        plane = 0;
        py = it / (4 * G);
        const int rem = it % (4 * G);
        k = rem >> 2;
        px = (rem & 3) * 4;
    } else {
        int c = it - LUMA;
        plane = c < CPL ? 1 : 2;
        c = c < CPL ? c : c - CPL;
        py = c / (G * CPR);
        const int rem = c % (G * CPR);
        k = rem / CPR;
        px = (rem % CPR) * 4;
    }
}

// select the k-th of G wave-uniform values (k lane-varying, G <= 4)
template <int G, class T>
__device__ __forceinline__ T pick(const T (&v)[G], int k) {
    T r = v[0];
#pragma unroll
    for (int i = 1; i < G; i++) r = (k == i) ? v[i] : r;
    return r;
}

// Raw reference words for one 4-pixel item in one direction: rows Y and Y+step, two aligned
// dwords each (the second row only when the vector is vertically half-pel).
struct Tap {
    uint32_t w0, w1, w2, w3;
};

template <int CF>
__device__ __forceinline__ void tap_geometry(uint32_t mvw, int plane, int gx, int py, int mby_base, bool field,
                                             int fs, int stride, int ph, int& off0, int& off1, int& sh, int& hxy) {
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
    } else {  // field MC (mb_decoder.cpp:229-236): row 2q + field_select, vector r = py & 1
        Y = mby_base + fs + 2 * ((py >> 1) + (mvy >> 1));
        step = 2;
    }
    // clamp into the plane: out-of-contract vectors can never fault (inactive in contract)
    const int Xc = min(max(X, 0), stride - 4);
    const int Y0 = min(max(Y, 0), ph - 1);
    const int Y1 = min(max(Y + step, 0), ph - 1);
    off0 = Y0 * stride + (Xc & ~3);
    off1 = Y1 * stride + (Xc & ~3);
    sh = (Xc & 3) * 8;
    hxy = (mvx & 1) | ((mvy & 1) << 1);
}

__device__ __forceinline__ Tap issue_tap(const uint8_t* __restrict__ plane_base, int off0, int off1, int hxy) {
    Tap t;
    const uint32_t* r0 = (const uint32_t*)(plane_base + off0);
    t.w0 = r0[0];
    t.w1 = r0[1];
    if (hxy & 2) {
        const uint32_t* r1 = (const uint32_t*)(plane_base + off1);
        t.w2 = r1[0];
        t.w3 = r1[1];
    } else {
        t.w2 = t.w3 = 0;
    }
    return t;
}

// cascaded half-pel average (mc_sse2.hpp:5-39 == mc_c.hpp:15)
__device__ __forceinline__ uint32_t finish_tap(const Tap& t, int sh, int hxy) {
    const uint64_t v0 = (((uint64_t)t.w1 << 32) | t.w0) >> sh;
    const uint32_t A = (uint32_t)v0, B = (uint32_t)(v0 >> 8);
    if (!(hxy & 2)) return (hxy & 1) ? avg4(A, B) : A;
    const uint64_t v1 = (((uint64_t)t.w3 << 32) | t.w2) >> sh;
    const uint32_t C = (uint32_t)v1, D = (uint32_t)(v1 >> 8);
    return (hxy & 1) ? avg4(avg4(A, B), avg4(C, D)) : avg4(A, C);
}

// Per-MB wave-uniform state of the group
template <int G>
struct Group {
    uint32_t mbx[G], mby[G], flags[G], cbp[G], qs[G], mv[4][G];  // mv[r*2+s][k]
    int slot_base[G];
    int coef_rel[G];  // first coefficient word of MB k, relative to the group's first
    int nslots, ncoef;
    uint32_t coef0;
};

template <int CF, int G, int ABL = 0>
__global__ __launch_bounds__(256) void recon_kernel(const mp2vg_picture_t* __restrict__ pics,
                                                    const uint32_t* __restrict__ mbrec,
                                                    const uint32_t* __restrict__ coefs,
                                                    const SliceDesc* __restrict__ slices,
                                                    uint8_t* __restrict__ pool, const Geo geo,
                                                    const uint32_t slice_base, const uint32_t nslices) {
    using F = Fmt<CF>;
    using RL = ResLayout<CF>;
    constexpr int NB = F::NB;
    constexpr int MAXS = G * NB;                     // coded-block slots per group
    constexpr int NIT = G * F::ITEMS;                // 4-pixel items per group
    constexpr int IPL = (NIT + 63) / 64;             // items per lane
    __shared__ __attribute__((aligned(16))) short s_blk[WAVES][MAXS][64];  // coef raster -> pass-1 out
    __shared__ __attribute__((aligned(16))) short s_res[WAVES][G][RL::SIZE];
    __shared__ int s_par[WAVES][MAXS];
    __shared__ uint8_t s_map[WAVES][MAXS];  // slot -> k*16 + b
    __shared__ uint8_t s_W[4][64];
    __shared__ uint8_t s_scan[64];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // XCD-aware mapping: consecutive slices (rows of one picture) share an XCD's L2
    // (bijective: XCD x = b % 8 owns the contiguous range [x*q + min(x, r), ...) of q or q+1 slices)
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
    for (int i = lane; i < MAXS; i += 64) s_par[wave][i] = 0;
    __syncthreads();

    uint8_t* const dst_slot = pool + (uint64_t)pic->dst_slot * geo.slot_bytes;
    const uint8_t* const ref_fwd = pool + (uint64_t)(pic->fwd_slot < 0 ? pic->dst_slot : pic->fwd_slot) * geo.slot_bytes;
    const uint8_t* const ref_bwd = pool + (uint64_t)(pic->bwd_slot < 0 ? pic->dst_slot : pic->bwd_slot) * geo.slot_bytes;

    const uint32_t mb_end = sd.mb_begin + sd.mb_count;
    for (uint32_t g0 = sd.mb_begin + wave * G; g0 < mb_end; g0 += WAVES * G) {
        // ---- group records (scalar loads; the MB array is padded by G records) ----
        const int ng = min((int)(mb_end - g0), G);
        Group<G> S;
        int sb = 0, cr = 0;
        const uint32_t* rp = mbrec + (size_t)g0 * 8;
        S.coef0 = rp[3];
#pragma unroll
        for (int k = 0; k < G; k++) {
            const uint32_t r0 = rp[k * 8 + 0], r1 = rp[k * 8 + 1], r2 = rp[k * 8 + 2];
            const bool live = k < ng;
            S.mbx[k] = r0 & 0xffff;
            S.mby[k] = r0 >> 16;
            S.flags[k] = live ? (r1 & 0xffff) : (uint32_t)MP2VG_MB_INTRA;
            S.cbp[k] = live ? ((r1 >> 16) & ((1u << NB) - 1)) : 0u;
            S.qs[k] = r2 & 0xff;
            S.slot_base[k] = sb;
            S.coef_rel[k] = cr;
            sb += __builtin_popcount(S.cbp[k]);
            cr += live ? (int)(r2 >> 16) : 0;
#pragma unroll
            for (int q = 0; q < 4; q++) S.mv[q][k] = rp[k * 8 + 4 + q];
        }
        S.nslots = sb;
        S.ncoef = cr;

        // ---- A. first 64 coefficient words (contiguous for the group; host-validated) ----
        const uint32_t cw0 = lane < S.ncoef ? coefs[S.coef0 + lane] : 0u;

        // ---- B. issue the MC loads of every item this lane owns (consumed in stage F) ----
        Tap tf[IPL], tb[IPL];
#pragma unroll
        for (int j = 0; j < IPL; j++) {
            const int it = lane + 64 * j;
            int k, plane, px, py;
            item_coords<CF, G>(it < NIT ? it : 0, k, plane, px, py);
            const uint32_t fl = pick<G>(S.flags, k);
            const bool intra = (fl & MP2VG_MB_INTRA) || it >= NIT || (ABL & 2);
            const bool bwd = fl & MP2VG_MB_BWD;
            const bool fwd = !intra && ((fl & MP2VG_MB_FWD) || !bwd);
            const bool field = fl & MP2VG_MB_FIELD_MC;
            const int pw = plane == 0 ? 16 : F::CW;
            const int phm = plane == 0 ? 16 : F::CH;
            const int gx = (int)pick<G>(S.mbx, k) * pw + px;
            const int mbyb = (int)pick<G>(S.mby, k) * phm;
            const int r = field ? (py & 1) : 0;
            const int stride = geo.stride[plane];
            tf[j] = Tap{0, 0, 0, 0};
            tb[j] = Tap{0, 0, 0, 0};
            if (fwd) {
                uint32_t mvw = (r ? pick<G>(S.mv[2], k) : pick<G>(S.mv[0], k));
                int o0, o1, sh, hxy;
                tap_geometry<CF>(mvw, plane, gx, py, mbyb, field, (fl >> (8 + 2 * r)) & 1, stride, geo.ph[plane], o0, o1, sh, hxy);
                tf[j] = issue_tap(ref_fwd + geo.plane_off[plane], o0, o1, hxy);
            }
            if (!intra && bwd) {
                uint32_t mvw = (r ? pick<G>(S.mv[3], k) : pick<G>(S.mv[1], k));
                int o0, o1, sh, hxy;
                tap_geometry<CF>(mvw, plane, gx, py, mbyb, field, (fl >> (9 + 2 * r)) & 1, stride, geo.ph[plane], o0, o1, sh, hxy);
                tb[j] = issue_tap(ref_bwd + geo.plane_off[plane], o0, o1, hxy);
            }
        }

        // ---- C. slot map + dequant/mismatch parity (parse_block, mb_decoder.cpp:74-155) ----
        if (lane < MAXS) {
            const int k = lane / NB, bb = lane % NB;
            const uint32_t cbpk = pick<G>(S.cbp, k);
            if (cbpk & (1u << bb)) s_map[wave][pick<G>(S.slot_base, k) + __builtin_popcount(cbpk & ((1u << bb) - 1))] = (uint8_t)(k * 16 + bb);
        }
        for (int k0 = 0; k0 < ((ABL & 4) ? 0 : S.ncoef); k0 += 64) {
            const int w_idx = k0 + lane;
            const uint32_t w = k0 == 0 ? cw0 : (w_idx < S.ncoef ? coefs[S.coef0 + w_idx] : 0u);
            if (w_idx >= S.ncoef) continue;
            int k = 0;
#pragma unroll
            for (int i = 1; i < G; i++) k += (w_idx >= S.coef_rel[i]) ? 1 : 0;
            const uint32_t cbpk = pick<G>(S.cbp, k);
            const int bb = (w >> 22) & 15;
            if (bb >= NB || !(cbpk & (1u << bb))) continue;  // host validation rejects these
            const int slot = pick<G>(S.slot_base, k) + __builtin_popcount(cbpk & ((1u << bb) - 1));
            const bool intra = pick<G>(S.flags, k) & MP2VG_MB_INTRA;
            const int qs = (int)pick<G>(S.qs, k);
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
            if (v & 1) atomicXor(&s_par[wave][slot], 1);
        }
        wave_sync();
        for (int s = lane; s < S.nslots; s += 64) {  // qfs[63] ^= !(sum & 1)   (:150-152)
            s_blk[wave][s][63] ^= (short)((s_par[wave][s] & 1) ^ 1);
            s_par[wave][s] = 0;
        }
        wave_sync();

        // ---- D. IDCT pass 1 (idct_sse2.hpp:102-103): lane (slot, v) transforms coefficient row v
        //         over u; output transposed IN PLACE ([x][v]) — the whole 8-lane block is read by
        //         one ds_read instruction before any lane writes.
        for (int t = lane; t < ((ABL & 1) ? 0 : S.nslots * 8); t += 64) {
            const int slot = t >> 3, v = t & 7;
            short s[8];
            const uint4 row = *(const uint4*)&s_blk[wave][slot][v * 8];
            s[0] = (short)(row.x & 0xffff); s[1] = (short)(row.x >> 16);
            s[2] = (short)(row.y & 0xffff); s[3] = (short)(row.y >> 16);
            s[4] = (short)(row.z & 0xffff); s[5] = (short)(row.z >> 16);
            s[6] = (short)(row.w & 0xffff); s[7] = (short)(row.w >> 16);
            idct_1d(s);
#pragma unroll
            for (int x = 0; x < 8; x++) s_blk[wave][slot][x * 8 + v] = s[x];
        }
        wave_sync();
        // pass 2 (:104-108): lane (slot, x) transforms column x over v; >>6 -> residual image in
        // the MB's dct_type placement (:166-196); the block area is zeroed for the next group
        for (int t = lane; t < ((ABL & 1) ? 0 : S.nslots * 8); t += 64) {
            const int slot = t >> 3, x = t & 7;
            short s[8];
            const uint4 row = *(const uint4*)&s_blk[wave][slot][x * 8];
            *(uint4*)&s_blk[wave][slot][x * 8] = make_uint4(0, 0, 0, 0);
            s[0] = (short)(row.x & 0xffff); s[1] = (short)(row.x >> 16);
            s[2] = (short)(row.y & 0xffff); s[3] = (short)(row.y >> 16);
            s[4] = (short)(row.z & 0xffff); s[5] = (short)(row.z >> 16);
            s[6] = (short)(row.w & 0xffff); s[7] = (short)(row.w >> 16);
            idct_1d(s);
            const int kb = s_map[wave][slot];
            const int k = kb >> 4, bb = kb & 15;
            const bool dctf = pick<G>(S.flags, k) & MP2VG_MB_DCT_FIELD;
            int plane, x0, y0, ys;
            block_origin<CF>(bb, dctf, plane, x0, y0, ys);
            short* res = &s_res[wave][k][RL::base(plane)];
            const int rw = RL::width(plane);
#pragma unroll
            for (int y = 0; y < 8; y++) res[(y0 + y * ys) * rw + x0 + x] = (short)(s[y] >> 6);
        }
        wave_sync();

        // ---- E. prediction (+ residual, clamp) and one 4-byte store per item ----
#pragma unroll
        for (int j = 0; j < IPL; j++) {
            const int it = lane + 64 * j;
            if (it >= NIT) continue;
            int k, plane, px, py;
            item_coords<CF, G>(it, k, plane, px, py);
            if (k >= ng) continue;
            const uint32_t fl = pick<G>(S.flags, k);
            const bool intra = fl & MP2VG_MB_INTRA;
            const bool bwd = fl & MP2VG_MB_BWD;
            const bool fwd = !intra && ((fl & MP2VG_MB_FWD) || !bwd);
            const bool field = fl & MP2VG_MB_FIELD_MC;
            const int pw = plane == 0 ? 16 : F::CW;
            const int phm = plane == 0 ? 16 : F::CH;
            const int mbx = (int)pick<G>(S.mbx, k), mby = (int)pick<G>(S.mby, k);
            const int stride = geo.stride[plane];
            const int r = field ? (py & 1) : 0;
            uint32_t pred = 0;
            if (!intra) {
                uint32_t pf = 0, pb = 0;
                if (fwd) {
                    int o0, o1, sh, hxy;
                    tap_geometry<CF>((r ? pick<G>(S.mv[2], k) : pick<G>(S.mv[0], k)), plane, mbx * pw + px, py, mby * phm,
                                     field, (fl >> (8 + 2 * r)) & 1, stride, geo.ph[plane], o0, o1, sh, hxy);
                    pf = finish_tap(tf[j], sh, hxy);
                }
                if (bwd) {
                    int o0, o1, sh, hxy;
                    tap_geometry<CF>((r ? pick<G>(S.mv[3], k) : pick<G>(S.mv[1], k)), plane, mbx * pw + px, py, mby * phm,
                                     field, (fl >> (9 + 2 * r)) & 1, stride, geo.ph[plane], o0, o1, sh, hxy);
                    pb = finish_tap(tb[j], sh, hxy);
                }
                pred = (fwd && bwd) ? avg4(pf, pb) : (fwd ? pf : pb);  // mc_sse2.hpp:78-84
            }
            const int bb = block_of<CF>(plane, px, py, fl & MP2VG_MB_DCT_FIELD);
            uint32_t out = pred;
            if (pick<G>(S.cbp, k) & (1u << bb)) {  // put: packus(res); add: packus(adds(pred,res))
                const uint2 rr = *(const uint2*)&s_res[wave][k][RL::base(plane) + py * RL::width(plane) + px];
                int q0 = (int)(pred & 255) + (short)(rr.x & 0xffff);
                int q1 = (int)((pred >> 8) & 255) + (short)(rr.x >> 16);
                int q2 = (int)((pred >> 16) & 255) + (short)(rr.y & 0xffff);
                int q3 = (int)(pred >> 24) + (short)(rr.y >> 16);
                q0 = min(max(q0, 0), 255);
                q1 = min(max(q1, 0), 255);
                q2 = min(max(q2, 0), 255);
                q3 = min(max(q3, 0), 255);
                out = (uint32_t)q0 | ((uint32_t)q1 << 8) | ((uint32_t)q2 << 16) | ((uint32_t)q3 << 24);
            }
            if (ABL & 8) asm volatile("" ::"v"(out)); else *(uint32_t*)(dst_slot + geo.plane_off[plane] + (size_t)(mby * phm + py) * stride + mbx * pw + px) = out;
        }
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

constexpr int kGroup = 2;

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
    case v: hipLaunchKernelGGL((recon_kernel<1, kGroup, v>), grid, block, 0, stream, a.pics, mb, a.coefs, a.slices, a.pool, g, a.slice_base, a.nslices); break;
        switch (ablate) {
            ABL_CASE(1) ABL_CASE(2) ABL_CASE(3) ABL_CASE(4) ABL_CASE(8) ABL_CASE(15)
        default: return hipErrorInvalidValue;
        }
#undef ABL_CASE
        return hipGetLastError();
    }
    switch (cf) {
    case 1: hipLaunchKernelGGL((recon_kernel<1, kGroup>), grid, block, 0, stream, a.pics, mb, a.coefs, a.slices, a.pool, g, a.slice_base, a.nslices); break;
    case 2: hipLaunchKernelGGL((recon_kernel<2, kGroup>), grid, block, 0, stream, a.pics, mb, a.coefs, a.slices, a.pool, g, a.slice_base, a.nslices); break;
    case 3: hipLaunchKernelGGL((recon_kernel<3, kGroup>), grid, block, 0, stream, a.pics, mb, a.coefs, a.slices, a.pool, g, a.slice_base, a.nslices); break;
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
