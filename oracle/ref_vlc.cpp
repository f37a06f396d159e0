// Test-infrastructure driver (ours): runs the REAL reference Annex B VLC decoders on every code of
// the reference's own code tables, followed by random suffixes, and records what they decode and
// how many bits they consume -- the data of the reference's VLC conformance test
// (test/gtest/cavlc/cavlc_test.cpp:25-88: every table entry, 100 random suffixes, value and
// consumed length checked), written out so our host parser can be pinned to it.
//
//   decoders: reference src/core/mp2v_vlc_dec.hpp:36-267 (templates over the bit reader)
//   tables:   reference src/core/mp2v_luts.hpp (compiled into mp2v_vlc.o)
//
// usage: ref_vlc <out> [suffixes_per_entry=32] [seed=1729]
//   out: records of { int32 table, entry; uint64 bits (MSB first: code, then suffix);
//                     int32 value, aux, consumed, code_len }
//   table ids (tests/golden/make_vlc_vectors.py): 0 MBA B.1 (get_macroblock_address_increment_lut),
//   10 MBA B.1 (get_macroblock_address_increment), 1/2/3 macroblock_type I/P/B B.2-B.4,
//   4 coded_block_pattern B.9, 5 motion_code B.10, 11 dmvector B.11, 6/7 dct_dc_size luma/chroma
//   B.12/B.13, 8/9 DCT coefficients B.14/B.15 (value = run, aux = level, unsigned: the sign bit
//   is read by the caller, mb_decoder.cpp:74-155).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "core/mp2v_vlc.h"

// The decoders are templates over a reader with get_next_bits / read_next_bits / skip_bits
// (reference bitstream.h:45-59); this one reads a 64-bit window and counts what is consumed,
// like the gtest's generator reader (cavlc_test.cpp:28-40 checks get_fullness() == 0).
struct window_reader {
    uint64_t w = 0;
    int pos = 0;
    uint32_t get_next_bits(int len) {
        if (!len) return 0;
        return (uint32_t)((w << pos) >> (64 - len));
    }
    uint32_t read_next_bits(int len) {
        uint32_t v = get_next_bits(len);
        pos += len;
        return v;
    }
    void skip_bits(int len) { pos += len; }
};

DEFINE_CAVLC_METHODS(window_reader)

struct rec {
    int32_t table, entry;
    uint64_t bits;
    int32_t value, aux, consumed, code_len;
};

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s out [suffixes] [seed]\n", argv[0]);
        return 2;
    }
    const int nsuf = argc > 2 ? atoi(argv[2]) : 32;
    std::mt19937_64 rng(argc > 3 ? strtoull(argv[3], nullptr, 10) : 1729);
    std::vector<rec> out;
    auto run = [&](int table, int entry, vlc_t code, auto decode) {
        for (int k = 0; k < nsuf; k++) {
            window_reader r;
            const uint64_t suffix = rng();
            r.w = ((uint64_t)code.value << (64 - code.len)) | (suffix >> code.len);
            rec x{table, entry, r.w, 0, 0, 0, code.len};
            decode(r, x);
            x.consumed = r.pos;
            out.push_back(x);
        }
    };
    for (int i = 1; i <= 33; i++) {
        run(0, i, macroblock_address_increment_to_vlc[i],
            [](window_reader& r, rec& x) { x.value = get_macroblock_address_increment_lut(&r); });
        run(10, i, macroblock_address_increment_to_vlc[i],
            [](window_reader& r, rec& x) { x.value = get_macroblock_address_increment(&r); });
    }
    for (int pct = 1; pct <= 3; pct++) {
        const macroblock_type_vlc_t* t = pct == 1 ? i_macroblock_type : (pct == 2 ? p_macroblock_type : b_macroblock_type);
        const int n = pct == 1 ? 2 : (pct == 2 ? 7 : 11);
        for (int i = 0; i < n; i++)
            run(pct, i, t[i].vlc, [pct](window_reader& r, rec& x) { x.value = get_macroblock_type(&r, pct); });
    }
    for (int i = 0; i < 64; i++)
        run(4, i, coded_block_pattern_to_vlc[i], [](window_reader& r, rec& x) { x.value = get_coded_block_pattern(&r); });
    for (int i = 0; i < 33; i++)
        run(5, i, motion_code_to_vlc[i], [](window_reader& r, rec& x) { x.value = get_motion_code(&r); });
    for (int i = 0; i < 3; i++)
        run(11, i, dmvector_to_vlc[i], [](window_reader& r, rec& x) { x.value = get_dmvector(&r); });
    for (int i = 0; i < 12; i++) {
        run(6, i, dct_size_luminance_to_vlc[i], [](window_reader& r, rec& x) { x.value = get_dct_size_luminance(&r); });
        run(7, i, dct_size_chrominance_to_vlc[i],
            [](window_reader& r, rec& x) { x.value = get_dct_size_chrominance(&r); });
    }
    for (int i = 0; i < 111; i++) {
        run(8, i, coeff_zero_vlc[i].vlc, [](window_reader& r, rec& x) {
            coeff_t c = get_coeff_zero(&r);
            x.value = c.run;
            x.aux = c.level;
        });
        run(9, i, coeff_one_vlc[i].vlc, [](window_reader& r, rec& x) {
            coeff_t c = get_coeff_one(&r);
            x.value = c.run;
            x.aux = c.level;
        });
    }
    FILE* f = fopen(argv[1], "wb");
    if (!f) {
        perror(argv[1]);
        return 1;
    }
    fwrite(out.data(), sizeof(rec), out.size(), f);
    fclose(f);
    printf("{\"records\": %zu}\n", out.size());
    return 0;
}
