/*
 * mp2v_oracle.c — TEST INFRASTRUCTURE ONLY (see mp2v_oracle.h).
 *
 * A plain-C restatement of the reference (fxslava/tiny_mp2v_dec) reconstruct path, x86 build:
 *   - IDCT: idct_sse2.hpp:7-120 (16-bit saturating AAN; horizontal-frequency pass first,
 *     transpose, second pass, srai 6, packus put / adds+packus add)
 *   - MC:   mc_c.hpp:3-87 (== mc_sse2.hpp:5-153; cascaded half-pel average)
 *   - dequant + mismatch: mb_decoder.cpp:74-155 (parse_block), DC :46-72 / :160
 *   - block placement and matrix choice: mb_decoder.cpp:166-196
 *   - MC dispatch: mb_decoder.cpp:198-339
 *   - frame layout: decoder.cpp:44-77, MB row pointers decoder.cpp:89-105
 * operating on the record stream of include/mp2vg.h instead of a bitstream.
 */
#include "mp2v_oracle.h"

#include <string.h>

/* scan position -> raster index (row = vertical frequency), zig-zag / alternate (ISO 13818-2
 * 7.3; the reference's g_shuffle, scan_c.cpp:41-57).  The reference stores QFS transposed:
 * g_scan_trans[a][i] = transpose(raster) (scan_c.cpp:4-21). */
static const uint8_t k_scan_raster[2][64] = {
    {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
     41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
     30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63},
    {0,  8,  16, 24, 1,  9,  2,  10, 17, 25, 32, 40, 48, 56, 57, 49, 41, 33, 26, 18, 3,  11,
     4,  12, 19, 27, 34, 42, 50, 58, 35, 43, 51, 59, 20, 28, 5,  13, 6,  14, 21, 29, 36, 44,
     52, 60, 37, 45, 53, 61, 22, 30, 7,  15, 23, 31, 38, 46, 54, 62, 39, 47, 55, 63}};

static int scan_trans(int alt, int i) {
    int r = k_scan_raster[alt][i];
    return ((r & 7) << 3) | (r >> 3);
}

/* ---------------- geometry (decoder.cpp:44-68) ---------------- */
void oracle_geometry(int width, int height, int cf, oracle_geom_t* g) {
    memset(g, 0, sizeof(*g));
    g->width = width;
    g->height = height;
    g->chroma_format = cf;
    g->stride[0] = (width + 63) & ~63;
    g->pw[0] = width;
    g->ph[0] = height;
    if (cf == 3) {
        g->stride[1] = g->stride[0];
        g->pw[1] = width;
        g->ph[1] = height;
    } else {
        g->stride[1] = ((g->stride[0] >> 1) + 63) & ~63;
        g->pw[1] = width >> 1;
        g->ph[1] = (cf == 1) ? (height >> 1) : height;
    }
    g->stride[2] = g->stride[1];
    g->pw[2] = g->pw[1];
    g->ph[2] = g->ph[1];
    g->plane_off[0] = 0;
    g->plane_off[1] = (uint64_t)g->stride[0] * g->ph[0];
    g->plane_off[2] = g->plane_off[1] + (uint64_t)g->stride[1] * g->ph[1];
    g->slot_bytes = g->plane_off[2] + (uint64_t)g->stride[2] * g->ph[2];
}

/* ---------------- SSE2 IDCT, scalar (idct_sse2.hpp) ---------------- */
static int16_t sat16(int32_t v) { return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v)); }
static int16_t adds(int16_t a, int16_t b) { return sat16((int32_t)a + b); }       /* _mm_adds_epi16 */
static int16_t subs(int16_t a, int16_t b) { return sat16((int32_t)a - b); }       /* _mm_subs_epi16 */
static int16_t mulhi(int16_t a, int16_t c) { return (int16_t)(((int32_t)a * c) >> 16); } /* _mm_mulhi_epi16 */
static int16_t slli(int16_t a, int n) { return (int16_t)(uint16_t)((uint32_t)(uint16_t)a << n); } /* wraps */

static int16_t op0(int16_t s) { return adds(s, mulhi(s, 27145)); } /* idct_sse2.hpp:7-9 */
static int16_t op1(int16_t s) { return subs(s, mulhi(s, 30068)); } /* :11-13 */
static int16_t op3(int16_t s) { return adds(s, mulhi(s, 20090)); } /* :15-17 */
static int16_t op4(int16_t s) { return mulhi(s, 25079); }          /* :19-21 */

/* idct_sse2.hpp:23-65, one lane */
static void idct_1d(int16_t s[8]) {
    int16_t v15 = adds(slli(mulhi(s[0], 27145), 1), slli(s[0], 1));
    int16_t v26 = adds(mulhi(s[1], -5037), slli(s[1], 2));
    int16_t v21 = adds(mulhi(s[2], -19954), slli(s[2], 2));
    int16_t v28 = adds(slli(mulhi(s[3], -22089), 1), slli(s[3], 2));
    int16_t v16 = adds(slli(mulhi(s[4], 27145), 1), slli(s[4], 1));
    int16_t v25 = adds(mulhi(s[5], 14567), slli(s[5], 1));
    int16_t v22 = adds(slli(mulhi(s[6], 17391), 1), s[6]);
    int16_t v27 = slli(mulhi(s[7], 25570), 1);
    int16_t v19 = subs(v25, v28);
    int16_t v20 = subs(v26, v27);
    int16_t v23 = adds(v26, v27);
    int16_t v24 = adds(v25, v28);
    int16_t v7 = adds(v23, v24);
    int16_t v11 = adds(v21, v22);
    int16_t v13 = subs(v23, v24);
    int16_t v17 = subs(v21, v22);
    int16_t v8 = adds(v15, v16);
    int16_t v9 = subs(v15, v16);
    int16_t v18 = op4(subs(v19, v20));
    int16_t v12 = subs(v18, op3(v19));
    int16_t v14 = subs(op1(v20), v18);
    int16_t v6 = subs(slli(v14, 1), v7);
    int16_t v5 = subs(op0(v13), v6);
    int16_t v4 = adds(v5, slli(v12, 1));
    int16_t v10 = subs(op0(v17), v11);
    int16_t v0 = adds(v8, v11);
    int16_t v1 = adds(v9, v10);
    int16_t v2 = subs(v9, v10);
    int16_t v3 = subs(v8, v11);
    s[0] = adds(v0, v7);
    s[1] = adds(v1, v6);
    s[2] = adds(v2, v5);
    s[3] = subs(v3, v4);
    s[4] = adds(v3, v4);
    s[5] = subs(v2, v5);
    s[6] = subs(v1, v6);
    s[7] = subs(v0, v7);
}

/* inverse_dct_template<add> (idct_sse2.hpp:96-120): buffer[i] = row i of F; the SIMD pass
 * transforms across rows for every column (lane); transpose; pass again. */
void oracle_idct(const int16_t F[64], uint8_t* plane, int stride, int add) {
    int16_t buf[8][8], col[8];
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) buf[i][j] = F[i * 8 + j];
    for (int pass = 0; pass < 2; pass++) {
        for (int j = 0; j < 8; j++) {
            for (int i = 0; i < 8; i++) col[i] = buf[i][j];
            idct_1d(col);
            for (int i = 0; i < 8; i++) buf[i][j] = col[i];
        }
        if (pass == 0) { /* transpose_8x8_sse2 (:67-94) */
            for (int i = 0; i < 8; i++)
                for (int j = i + 1; j < 8; j++) {
                    int16_t t = buf[i][j];
                    buf[i][j] = buf[j][i];
                    buf[j][i] = t;
                }
        }
    }
    for (int i = 0; i < 8; i++) {
        uint8_t* row = plane + (ptrdiff_t)i * stride;
        for (int j = 0; j < 8; j++) {
            int16_t b = (int16_t)(buf[i][j] >> 6); /* _mm_srai_epi16(.., 6) */
            int16_t v = add ? adds((int16_t)row[j], b) : b;
            row[j] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); /* _mm_packus_epi16 */
        }
    }
}

/* ---------------- MC (mc_c.hpp; enum mc.h:4 MC_00, MC_10(vert), MC_01(horiz), MC_11) ------ */
static uint8_t mc_px(const uint8_t* src, int i, int stride, int type) {
    switch (type) {
    case 0: return src[i];
    case 1: return (uint8_t)((src[i] + src[i + 1] + 1) >> 1);            /* idx bit0: x half */
    case 2: return (uint8_t)((src[i] + src[i + stride] + 1) >> 1);       /* idx bit1: y half */
    default:
        return (uint8_t)((((src[i] + src[i + 1] + 1) >> 1) +
                          ((src[i + stride] + src[i + stride + 1] + 1) >> 1) + 1) >> 1);
    }
}

/* idx as the reference tables: pred: (mvx&1)|(mvy&1)<<1 (mb_decoder.cpp:253-255) applied to
 * src0; bidir: fx|fy<<1 (applied to src1 = fref) | bx<<2|by<<3 (src0 = bref)
 * (mb_decoder.cpp:208-210, call mc_bidir(dst, bref, fref) :240-248; table mc.cpp:18-25). */
void oracle_mc(uint8_t* dst, const uint8_t* src0, const uint8_t* src1, int stride, int width,
               int height, int bidir, int idx) {
    for (int y = 0; y < height; y++) {
        for (int x = 0; x < width; x++) {
            if (!bidir) {
                dst[x] = mc_px(src0, x, stride, idx & 3);
            } else {
                uint8_t a = mc_px(src0, x, stride, (idx >> 2) & 3);
                uint8_t b = mc_px(src1, x, stride, idx & 3);
                dst[x] = (uint8_t)((a + b + 1) >> 1);
            }
        }
        dst += stride;
        src0 += stride;
        if (src1) src1 += stride;
    }
}

/* ---------------- dequant + mismatch (parse_block, mb_decoder.cpp:74-155) ---------------- */
void oracle_dequant_block(const uint32_t* words, int n, const uint8_t W[64], int qs, int intra,
                          int alt, int16_t QFS[64]) {
    int sum = 0;
    memset(QFS, 0, 64 * sizeof(int16_t));
    for (int k = 0; k < n; k++) {
        uint32_t w = words[k];
        int level = MP2VG_COEF_LEVEL(w);
        int i = (int)MP2VG_COEF_POS(w);
        if (w & MP2VG_COEF_DC) { /* QFS[0] = dc_pred << (3 - prec), not in the sum (:160) */
            QFS[0] = (int16_t)level;
            continue;
        }
        int sign = level < 0 ? -1 : 0;
        int mag = level < 0 ? -level : level;
        if (w & MP2VG_COEF_FIRST1S) { /* :79-88 — unclamped, stored at qfs[0], in the sum */
            int16_t val = (int16_t)((3 * W[i] * qs) >> 5);
            QFS[i] = (int16_t)((val ^ sign) - sign);
            sum += QFS[i];
            continue;
        }
        int32_t val = intra ? (mag * W[i] * qs) >> 4 : ((2 * mag + 1) * W[i] * qs) >> 5;
        val = (val ^ sign) - sign;
        int16_t t = (int16_t)val; /* truncation to int16 BEFORE the clamp (:146) */
        if (t > 2047) t = 2047;
        if (t < -2048) t = -2048;
        QFS[scan_trans(alt, i)] = t;
        sum += t;
    }
    QFS[63] ^= (int16_t)((sum & 1) ^ 1); /* :150-152 */
}

/* ---------------- MC dispatch (mb_decoder.cpp:198-339) ---------------- */
typedef struct mb_ptrs {
    uint8_t* p[3][3]; /* [SRC/L0/L1][Y/U/V] at the MB origin */
} mb_ptrs_t;

static void chroma_scale(int cf, int plane, int* mvx, int* mvy) { /* :198-206 */
    if (plane > 0) {
        if (cf < 3) *mvx >>= 1; /* arithmetic shift: floor */
        if (cf < 2) *mvy >>= 1;
    }
}

static void mc_plane(const oracle_geom_t* g, const mp2vg_mb_t* mb, mb_ptrs_t* P, int plane,
                     int r, int field, int fwd, int bwd) {
    int cf = g->chroma_format;
    int stride = g->stride[plane];
    int st = field ? stride * 2 : stride;
    int w = (plane == 0 || cf == 3) ? 16 : 8;
    int h = (plane == 0 || cf != 1) ? 16 : 8;
    if (field) h >>= 1;
    uint8_t* dst = P->p[0][plane] + (field && r ? stride : 0);
    if (fwd && bwd) { /* mc_bidir_template :212-251 */
        int fx = mb->mv[r][0][0], fy = mb->mv[r][0][1];
        int bx = mb->mv[r][1][0], by = mb->mv[r][1][1];
        chroma_scale(cf, plane, &fx, &fy);
        chroma_scale(cf, plane, &bx, &by);
        int idx = (fx & 1) | ((fy & 1) << 1) | ((bx & 1) << 2) | ((by & 1) << 3);
        const uint8_t* fref = P->p[1][plane] + (fx >> 1) + (ptrdiff_t)(fy >> 1) * st;
        const uint8_t* bref = P->p[2][plane] + (bx >> 1) + (ptrdiff_t)(by >> 1) * st;
        if (field) {
            if (mb->flags & MP2VG_MB_FS_BIT(r, 0)) fref += stride;
            if (mb->flags & MP2VG_MB_FS_BIT(r, 1)) bref += stride;
        }
        oracle_mc(dst, bref, fref, st, w, h, 1, idx);
    } else { /* mc_unidir_template :257-289 (the 'else' branch of :329 is forward) */
        int s = (!fwd && bwd) ? 1 : 0;
        int mx = mb->mv[r][s][0], my = mb->mv[r][s][1];
        chroma_scale(cf, plane, &mx, &my);
        int idx = (mx & 1) | ((my & 1) << 1);
        const uint8_t* ref = P->p[s ? 2 : 1][plane] + (mx >> 1) + (ptrdiff_t)(my >> 1) * st;
        if (field && (mb->flags & MP2VG_MB_FS_BIT(r, s))) ref += stride;
        oracle_mc(dst, ref, NULL, st, w, h, 0, idx);
    }
}

/* ---------------- block placement (decode_transform_template :166-196) ---------------- */
static void block_origin(const oracle_geom_t* g, int b, int dct_field, int* plane, int* x,
                         int* y, int* ystep) {
    int cf = g->chroma_format;
    *ystep = 1;
    if (b < 4) {
        *plane = 0;
        *x = (b & 1) * 8;
        if (dct_field) {
            *y = b >> 1;
            *ystep = 2;
        } else {
            *y = (b >> 1) * 8;
        }
        return;
    }
    *plane = (b & 1) ? 2 : 1; /* even blocks Cb, odd Cr (:184-195) */
    int k = (b - 4) >> 1;     /* 0: blocks 4/5, 1: 6/7, 2: 8/9, 3: 10/11 */
    int fld = dct_field && cf != 1;
    *x = (k >= 2) ? 8 : 0;
    int lower = (k == 1 || k == 3);
    if (fld) {
        *y = lower ? 1 : 0;
        *ystep = 2;
    } else {
        *y = lower ? 8 : 0;
    }
}

int oracle_reconstruct(const oracle_geom_t* g, const mp2vg_picture_t* pics, int npics,
                       const mp2vg_mb_t* mbs, const uint32_t* coefs, uint8_t* pool, int nslots) {
    int cf = g->chroma_format;
    int nblocks = cf == 1 ? 6 : (cf == 2 ? 8 : 12);
    int cw = cf == 3 ? 16 : 8, ch = cf == 1 ? 8 : 16;
    for (int pi = 0; pi < npics; pi++) {
        const mp2vg_picture_t* pic = &pics[pi];
        if (pic->dst_slot < 0 || pic->dst_slot >= nslots) return -1;
        uint8_t* slot[3] = {pool + (uint64_t)pic->dst_slot * g->slot_bytes,
                            pic->fwd_slot >= 0 ? pool + (uint64_t)pic->fwd_slot * g->slot_bytes : NULL,
                            pic->bwd_slot >= 0 ? pool + (uint64_t)pic->bwd_slot * g->slot_bytes : NULL};
        int nmb = pic->mb_width * pic->mb_height;
        for (int m = 0; m < nmb; m++) {
            const mp2vg_mb_t* mb = &mbs[pic->mb_first + m];
            mb_ptrs_t P;
            for (int t = 0; t < 3; t++)
                for (int pl = 0; pl < 3; pl++) {
                    if (!slot[t]) {
                        P.p[t][pl] = NULL;
                        continue;
                    }
                    int mw = pl == 0 ? 16 : cw, mh = pl == 0 ? 16 : ch;
                    P.p[t][pl] = slot[t] + g->plane_off[pl] + (uint64_t)mb->y * mh * g->stride[pl] +
                                 (uint64_t)mb->x * mw;
                }
            int intra = mb->flags & MP2VG_MB_INTRA;
            if (!intra) {
                int fwd = !!(mb->flags & MP2VG_MB_FWD), bwd = !!(mb->flags & MP2VG_MB_BWD);
                if (!fwd && !bwd) fwd = 1; /* :329-337 */
                if ((fwd && !P.p[1][0]) || (bwd && !P.p[2][0])) return -1;
                int field = !!(mb->flags & MP2VG_MB_FIELD_MC);
                for (int r = 0; r < (field ? 2 : 1); r++)
                    for (int pl = 0; pl < 3; pl++) mc_plane(g, mb, &P, pl, r, field, fwd, bwd);
            }
            /* blocks: coefficient words are grouped by block in bitstream order */
            const uint32_t* w = coefs + mb->coef_off;
            int k = 0;
            for (int b = 0; b < nblocks; b++) {
                if (!(mb->cbp & (1u << b))) continue;
                int n = 0;
                while (k + n < mb->ncoef && (int)MP2VG_COEF_BLOCK(w[k + n]) == b) n++;
                int16_t QFS[64];
                int mat = (b < 6 ? 0 : 2) + (intra ? 0 : 1);
                oracle_dequant_block(w + k, n, pic->W[mat], mb->qscale, intra,
                                     pic->alternate_scan, QFS);
                k += n;
                int plane, x, y, ystep;
                block_origin(g, b, !!(mb->flags & MP2VG_MB_DCT_FIELD), &plane, &x, &y, &ystep);
                uint8_t* dst = P.p[0][plane] + (ptrdiff_t)y * g->stride[plane] + x;
                oracle_idct(QFS, dst, g->stride[plane] * ystep, !intra);
            }
            if (k != mb->ncoef) return -1;
        }
    }
    return 0;
}
