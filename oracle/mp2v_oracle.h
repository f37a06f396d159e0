/*
 * mp2v_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C) of the reference's macroblock reconstruct path, consuming the same
 * record stream the HIP kernels consume (include/mp2vg.h).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it, and only as the checker — the product library
 * never links it and has no CPU fallback.
 *
 * Parity pinned: tests/test_oracle_golden.py checks this oracle bit-exact against outputs of the
 * REAL reference (oracle/_ref, built from /root/reference by oracle/Makefile) — whole decoded
 * streams (tests/golden/streams/) and per-kernel vectors (tests/golden/idct_vectors.npz,
 * mc_vectors.npz).
 */
#ifndef MP2V_ORACLE_H
#define MP2V_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/mp2vg.h"

typedef struct oracle_geom {
    int width, height, chroma_format;
    int pw[3], ph[3], stride[3];
    uint64_t plane_off[3];
    uint64_t slot_bytes;
} oracle_geom_t;

void oracle_geometry(int width, int height, int chroma_format, oracle_geom_t* g);

/* Reconstruct the pictures in the given (decode) order into the frame pool `pool`
 * (nslots * g->slot_bytes bytes, slot layout from oracle_geometry).  Returns 0 or -1. */
int oracle_reconstruct(const oracle_geom_t* g, const mp2vg_picture_t* pics, int npics,
                       const mp2vg_mb_t* mbs, const uint32_t* coefs, uint8_t* pool, int nslots);

/* Per-kernel entry points (for the golden kernel vectors). */
void oracle_idct(const int16_t F[64], uint8_t* plane, int stride, int add);
void oracle_mc(uint8_t* dst, const uint8_t* src0, const uint8_t* src1, int stride, int width,
               int height, int bidir, int idx);
/* dequant + mismatch of one block's coefficient words into QFS (transposed raster) */
void oracle_dequant_block(const uint32_t* words, int n, const uint8_t W[64], int qscale,
                          int intra, int alt_scan, int16_t QFS[64]);
#endif
