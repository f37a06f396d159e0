// recon.hip — HIP kernels of the macroblock reconstruct path (see recon_kernel.h for the map to
// the reference).  Written for gfx950 only: wave64, LDS per wave, no CUDA-compat layer.
#include <hip/hip_runtime.h>
#include <stdint.h>

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

template <int CF>
__global__ __launch_bounds__(256) void recon_kernel(KArgs a) {
    using F = Fmt<CF>;
    constexpr int NB = F::NB;
    __shared__ __attribute__((aligned(16))) short s_coef[WAVES][NB][64];  // raster v*8+u
    __shared__ __attribute__((aligned(16))) short s_tmp[WAVES][NB][64];   // [x][v]
    __shared__ __attribute__((aligned(16))) short s_res[WAVES][3][16 * 16];
    __shared__ int s_par[WAVES][16];
    __shared__ uint8_t s_W[4][64];
    __shared__ uint8_t s_scan[64];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const SliceDesc sd = a.slices[a.slice_base + blockIdx.x];
    const mp2vg_picture_t* pic = a.pics + sd.pic;
    const int alt = pic->alternate_scan;

    // picture matrices + scan table into LDS
    if (tid < 64) {
        ((uint32_t*)s_W)[tid] = ((const uint32_t*)pic->W)[tid];
        s_scan[tid] = c_scan_raster[alt & 1][tid];
    }
    for (int i = lane; i < NB * 64 / 2; i += 64) ((uint32_t*)s_coef[wave])[i] = 0;
    if (lane < 16) s_par[wave][lane] = 0;
    __syncthreads();

    uint8_t* dst_slot = a.pool + (uint64_t)pic->dst_slot * a.slot_bytes;
    const uint8_t* ref_slot[2] = {
        a.pool + (uint64_t)(pic->fwd_slot < 0 ? pic->dst_slot : pic->fwd_slot) * a.slot_bytes,
        a.pool + (uint64_t)(pic->bwd_slot < 0 ? pic->dst_slot : pic->bwd_slot) * a.slot_bytes};

    const uint32_t mb_end = sd.mb_begin + sd.mb_count;
    for (uint32_t m = sd.mb_begin + wave; m < mb_end; m += WAVES) {
        const mp2vg_mb_t mb = a.mbs[m];
        const bool intra = mb.flags & MP2VG_MB_INTRA;
        const bool dctf = mb.flags & MP2VG_MB_DCT_FIELD;
        const uint32_t cbp = mb.cbp & ((1u << NB) - 1);
        const int qs = mb.qscale;

        // ---- 1. dequant + mismatch parity (parse_block, mb_decoder.cpp:74-155) ----
        for (int k = lane; k < mb.ncoef; k += 64) {
            const uint32_t w = a.coefs[mb.coef_off + k];
            const int b = (w >> 22) & 15;
            if (b >= NB || !(cbp & (1u << b))) continue;  // host validation rejects these
            const int i = (w >> 16) & 63;
            const int level = (short)(w & 0xffff);
            if (w & MP2VG_COEF_DC) {  // QFS[0] = dc << (3 - prec), outside the parity sum
                s_coef[wave][b][0] = (short)level;
                continue;
            }
            const int mat = (b < 6 ? 0 : 2) + (intra ? 0 : 1);
            const int Wi = s_W[mat][i];
            const int sign = level < 0 ? -1 : 0;
            const int mag = level < 0 ? -level : level;
            short v;
            int pos;
            if (w & MP2VG_COEF_FIRST1S) {  // (3*W*qs)>>5, unclamped (mb_decoder.cpp:79-88)
                short t = (short)((3 * Wi * qs) >> 5);
                v = (short)((t ^ sign) - sign);
                pos = i;  // stored at qfs[i] directly (i == 0)
                pos = ((pos & 7) << 3) | (pos >> 3);
            } else {
                int val = intra ? (mag * Wi * qs) >> 4 : ((2 * mag + 1) * Wi * qs) >> 5;
                val = (val ^ sign) - sign;
                short t = (short)val;  // int16 truncation before the clamp (:146)
                v = t > 2047 ? (short)2047 : (t < -2048 ? (short)-2048 : t);
                pos = s_scan[i];
            }
            s_coef[wave][b][pos] = v;
            if (v & 1) atomicXor(&s_par[wave][b], 1);
        }
        wave_sync();
        if (lane < NB && (cbp & (1u << lane))) {  // qfs[63] ^= !(sum & 1)   (:150-152)
            s_coef[wave][lane][63] ^= (short)((s_par[wave][lane] & 1) ^ 1);
            s_par[wave][lane] = 0;
        }
        wave_sync();

        // ---- 2. IDCT pass 1: lane (b, v) transforms coefficient row v over u ----
        for (int t = lane; t < NB * 8; t += 64) {
            const int b = t >> 3, v = t & 7;
            if (!(cbp & (1u << b))) continue;
            short s[8];
            uint4 row = *(const uint4*)&s_coef[wave][b][v * 8];
            *(uint4*)&s_coef[wave][b][v * 8] = make_uint4(0, 0, 0, 0);
            s[0] = (short)(row.x & 0xffff); s[1] = (short)(row.x >> 16);
            s[2] = (short)(row.y & 0xffff); s[3] = (short)(row.y >> 16);
            s[4] = (short)(row.z & 0xffff); s[5] = (short)(row.z >> 16);
            s[6] = (short)(row.w & 0xffff); s[7] = (short)(row.w >> 16);
            idct_1d(s);
#pragma unroll
            for (int x = 0; x < 8; x++) s_tmp[wave][b][x * 8 + v] = s[x];
        }
        wave_sync();
        // pass 2: lane (b, x) transforms column x over v; >>6 -> residual image
        for (int t = lane; t < NB * 8; t += 64) {
            const int b = t >> 3, x = t & 7;
            if (!(cbp & (1u << b))) continue;
            short s[8];
            uint4 row = *(const uint4*)&s_tmp[wave][b][x * 8];
            s[0] = (short)(row.x & 0xffff); s[1] = (short)(row.x >> 16);
            s[2] = (short)(row.y & 0xffff); s[3] = (short)(row.y >> 16);
            s[4] = (short)(row.z & 0xffff); s[5] = (short)(row.z >> 16);
            s[6] = (short)(row.w & 0xffff); s[7] = (short)(row.w >> 16);
            idct_1d(s);
            int plane, x0, y0, ys;
            block_origin<CF>(b, dctf, plane, x0, y0, ys);
#pragma unroll
            for (int y = 0; y < 8; y++) s_res[wave][plane][(y0 + y * ys) * 16 + x0 + x] = (short)(s[y] >> 6);
        }
        wave_sync();

        // ---- 3. MC + add/clip + store ----
        const bool fwd = (mb.flags & MP2VG_MB_FWD) || (!intra && !(mb.flags & MP2VG_MB_BWD));
        const bool bwd = mb.flags & MP2VG_MB_BWD;
        const bool field = mb.flags & MP2VG_MB_FIELD_MC;
        for (int it = lane; it < F::ITEMS; it += 64) {
            int plane, px, py;
            if (it < 64) {
                plane = 0;
                py = it >> 2;
                px = (it & 3) * 4;
            } else {
                int c = it - 64;
                constexpr int per_plane = (F::CW / 4) * F::CH;
                plane = c < per_plane ? 1 : 2;
                c = c < per_plane ? c : c - per_plane;
                py = c / (F::CW / 4);
                px = (c % (F::CW / 4)) * 4;
            }
            const int pw = plane == 0 ? 16 : F::CW;
            const int phm = plane == 0 ? 16 : F::CH;
            const int stride = a.stride[plane];
            const int gx = mb.x * pw + px;
            const int gy = mb.y * phm + py;
            uint32_t pred = 0;
            if (!intra) {
                uint32_t p2[2];
                int np = 0;
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    if (!(s == 0 ? fwd : bwd)) continue;
                    const int r = field ? (py & 1) : 0;
                    int mvx = mb.mv[r][s][0], mvy = mb.mv[r][s][1];
                    if (plane > 0) {  // apply_chroma_scale (mb_decoder.cpp:198-206)
                        if (CF < 3) mvx >>= 1;
                        if (CF < 2) mvy >>= 1;
                    }
                    const int X = gx + (mvx >> 1);
                    int Y, step;
                    if (!field) {
                        Y = gy + (mvy >> 1);
                        step = 1;
                    } else {
                        const int fs = (mb.flags >> (8 + 2 * r + s)) & 1;
                        Y = mb.y * phm + fs + 2 * ((py >> 1) + (mvy >> 1));
                        step = 2;
                    }
                    // clamp into the plane: never fault on out-of-contract vectors
                    const int Xc = min(max(X, 0), stride - 4);
                    const int Y0 = min(max(Y, 0), a.ph[plane] - 1);
                    const int Y1 = min(max(Y + step, 0), a.ph[plane] - 1);
                    const uint8_t* refp = ref_slot[s] + a.plane_off[plane];
                    uint32_t A, B;
                    load5(refp + (size_t)Y0 * stride + Xc, A, B);
                    uint32_t v;
                    const int hx = mvx & 1, hy = mvy & 1;
                    if (hy) {
                        uint32_t C, D;
                        load5(refp + (size_t)Y1 * stride + Xc, C, D);
                        v = hx ? avg4(avg4(A, B), avg4(C, D)) : avg4(A, C);
                    } else {
                        v = hx ? avg4(A, B) : A;
                    }
                    p2[np++] = v;
                }
                pred = np == 2 ? avg4(p2[0], p2[1]) : p2[0];
            }
            const int b = block_of<CF>(plane, px, py, dctf);
            uint32_t out;
            if (cbp & (1u << b)) {
                const uint2 rr = *(const uint2*)&s_res[wave][plane][py * 16 + px];
                int r0 = (short)(rr.x & 0xffff), r1 = (short)(rr.x >> 16);
                int r2 = (short)(rr.y & 0xffff), r3 = (short)(rr.y >> 16);
                int q0 = (int)(pred & 255) + r0, q1 = (int)((pred >> 8) & 255) + r1;
                int q2 = (int)((pred >> 16) & 255) + r2, q3 = (int)(pred >> 24) + r3;
                q0 = min(max(q0, 0), 255);
                q1 = min(max(q1, 0), 255);
                q2 = min(max(q2, 0), 255);
                q3 = min(max(q3, 0), 255);
                out = (uint32_t)q0 | ((uint32_t)q1 << 8) | ((uint32_t)q2 << 16) | ((uint32_t)q3 << 24);
            } else {
                out = pred;
            }
            *(uint32_t*)(dst_slot + a.plane_off[plane] + (size_t)gy * stride + gx) = out;
        }
        wave_sync();
    }
}

template __global__ void recon_kernel<1>(KArgs);
template __global__ void recon_kernel<2>(KArgs);
template __global__ void recon_kernel<3>(KArgs);

// 64-bit digest of a slot's visible planes: sum over rows of fnv1a(row) * (2*row_id + 1)
__global__ void digest_kernel(const uint8_t* pool, uint64_t slot_bytes, const int32_t* slots, int nslots,
                              uint64_t o0, uint64_t o1, uint64_t o2, int s0, int s1, int w0, int w1,
                              int h0, int h1, unsigned long long* out) {
    const int rows = h0 + 2 * h1;
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int si = gid / rows, row = gid % rows;
    if (si >= nslots) return;
    const uint8_t* base = pool + (uint64_t)slots[si] * slot_bytes;
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
    uint64_t h = 1469598103934665603ull;
    for (int x = 0; x < w; x++) {
        h ^= p[x];
        h *= 1099511628211ull;
    }
    atomicAdd(&out[si], (unsigned long long)(h * (uint64_t)(2 * row + 1)));
}

}  // namespace mp2vg

namespace mp2vg {

hipError_t launch_recon(int cf, const KArgs& a, hipStream_t stream) {
    dim3 grid(a.nslices), block(256);
    switch (cf) {
    case 1: hipLaunchKernelGGL(recon_kernel<1>, grid, block, 0, stream, a); break;
    case 2: hipLaunchKernelGGL(recon_kernel<2>, grid, block, 0, stream, a); break;
    case 3: hipLaunchKernelGGL(recon_kernel<3>, grid, block, 0, stream, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_digest(const uint8_t* pool, uint64_t slot_bytes, const int32_t* d_slots, int n,
                         const uint64_t off[3], const int32_t stride[3], const int32_t w[3],
                         const int32_t h[3], unsigned long long* d_out, hipStream_t stream) {
    int rows = h[0] + 2 * h[1];
    int total = rows * n;
    dim3 block(256), grid((total + 255) / 256);
    hipLaunchKernelGGL(digest_kernel, grid, block, 0, stream, pool, slot_bytes, d_slots, n, off[0], off[1],
                       off[2], stride[0], stride[1], w[0], w[1], h[0], h[1], d_out);
    return hipGetLastError();
}

}  // namespace mp2vg
