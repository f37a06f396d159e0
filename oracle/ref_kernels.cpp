// Test-infrastructure driver (ours): runs the REAL reference x86 kernels on vectors we supply,
// so the golden fixtures under tests/golden/ come from the reference itself.
//
//  idct: reference idct_sse2.hpp:96-120 inverse_dct_template<false> (put) and <true> (add)
//  mc  : reference mc.cpp:4-25 tables mc_pred_16xh/8xh, mc_bidir_16xh/8xh (-> mc_sse2.hpp)
//
// usage: ref_kernels idct <in> <out>
//          in : N records of { int16 F[64] (QFS layout, transposed raster); uint8 pred[64] }
//          out: N records of { uint8 put[64]; uint8 add[64] }   (8x8, stride 8)
//        ref_kernels mc <in> <out>
//          in : int32 hdr[4] = {stride, rows, ncases, 0}; uint8 planeA[stride*rows];
//               uint8 planeB[stride*rows];
//               ncases x int32 {bidir, width(8|16), height, idx, offA, offB, 0, 0}
//          out: ncases x uint8 dst[stride*height] (dst pre-filled with 0xA5)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "core/idct_sse2.hpp"
#include "core/mc.h"

static std::vector<uint8_t> slurp(const char* p) {
    FILE* f = fopen(p, "rb");
    if (!f) { perror(p); exit(1); }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<uint8_t> v(n);
    if (fread(v.data(), 1, n, f) != (size_t)n) { perror("read"); exit(1); }
    fclose(f);
    return v;
}

int main(int argc, char** argv) {
    if (argc != 4) { fprintf(stderr, "usage: %s idct|mc in out\n", argv[0]); return 2; }
    std::vector<uint8_t> in = slurp(argv[2]);
    std::vector<uint8_t> out;
    if (!strcmp(argv[1], "idct")) {
        size_t n = in.size() / 192;
        out.resize(n * 128);
        for (size_t k = 0; k < n; k++) {
            ALIGN(32) int16_t F[64];
            ALIGN(32) uint8_t put[64];
            ALIGN(32) uint8_t add[64];
            memcpy(F, &in[k * 192], 128);
            memcpy(add, &in[k * 192 + 128], 64);
            memset(put, 0, 64);
            inverse_dct_template<false>(put, F, 8);
            memcpy(F, &in[k * 192], 128);  // the SSE2 routine takes F by pointer; keep it pristine
            inverse_dct_template<true>(add, F, 8);
            memcpy(&out[k * 128], put, 64);
            memcpy(&out[k * 128 + 64], add, 64);
        }
    } else if (!strcmp(argv[1], "mc")) {
        const int32_t* hdr = (const int32_t*)in.data();
        int stride = hdr[0], rows = hdr[1], ncases = hdr[2];
        const uint8_t* A = in.data() + 16;
        const uint8_t* B = A + (size_t)stride * rows;
        const int32_t* cases = (const int32_t*)(B + (size_t)stride * rows);
        std::vector<uint8_t> pa(A, A + (size_t)stride * rows), pb(B, B + (size_t)stride * rows);
        for (int c = 0; c < ncases; c++) {
            const int32_t* cs = cases + c * 8;
            int bidir = cs[0], width = cs[1], height = cs[2], idx = cs[3];
            std::vector<uint8_t> dst((size_t)stride * height + 16, 0xA5);
            if (!bidir) {
                mc_pred_func_t f = (width == 16 ? mc_pred_16xh : mc_pred_8xh)[idx];
                f(dst.data(), pa.data() + cs[4], stride, height);
            } else {
                mc_bidir_func_t f = (width == 16 ? mc_bidir_16xh : mc_bidir_8xh)[idx];
                f(dst.data(), pa.data() + cs[4], pb.data() + cs[5], stride, height);
            }
            out.insert(out.end(), dst.begin(), dst.begin() + (size_t)stride * height);
        }
    } else {
        fprintf(stderr, "unknown mode %s\n", argv[1]);
        return 2;
    }
    FILE* f = fopen(argv[3], "wb");
    fwrite(out.data(), 1, out.size(), f);
    fclose(f);
    return 0;
}
