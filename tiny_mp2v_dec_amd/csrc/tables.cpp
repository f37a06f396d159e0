#include <chrono>
#include <cstdio>
#include <cstdlib>
// tables.cpp — decode LUTs built once from the Annex B code lists in vlc_tables.h, scan tables,
// error plumbing shared by the whole library.
#include <mutex>
#include <string>

#include "syntax.h"

namespace mp2vg {

// scan position -> raster index (v*8+u): zig-zag and alternate scan (ISO 13818-2 7.3,
// reference scan_c.cpp:41-57 g_shuffle)
const uint8_t kScanRaster[2][64] = {
    {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
     41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
     30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63},
    {0,  8,  16, 24, 1,  9,  2,  10, 17, 25, 32, 40, 48, 56, 57, 49, 41, 33, 26, 18, 3,  11,
     4,  12, 19, 27, 34, 42, 50, 58, 35, 43, 51, 59, 20, 28, 5,  13, 6,  14, 21, 29, 36, 44,
     52, 60, 37, 45, 53, 61, 22, 30, 7,  15, 23, 31, 38, 46, 54, 62, 39, 47, 55, 63}};

template <int N>
static void add_list(VlcLut& l, const vlc_code (&codes)[N]) {
    for (int i = 0; i < N; i++) l.add(codes[i].bits, i);
}

void CoefLut::add(const char* bits, int run, int level, int kind) {
    const int len = (int)strlen(bits);
    for (int sign = 0; sign < (kind == NORMAL ? 2 : 1); sign++) {
        uint32_t code = 0;
        for (int i = 0; i < len; i++) code = (code << 1) | (bits[i] == '1');
        int n = len;
        int lv = level;
        if (kind == NORMAL) {
            code = (code << 1) | (uint32_t)sign;
            n++;
            lv = sign ? -level : level;
        }
        if (n <= L1) {
            const uint32_t lo = code << (L1 - n), hi = (code + 1) << (L1 - n);
            for (uint32_t v = lo; v < hi; v++) l1[v] = pack(n, run, lv, kind);
        } else {
            const uint32_t pre = code >> (n - L1);
            uint32_t& e = l1[pre];
            if (((e >> 23) & 3) != SUB) {
                const uint32_t idx = (uint32_t)(l2.size() / 128);
                l2.resize(l2.size() + 128, 0);
                e = pack(0, 0, 0, SUB) | (idx << 5);
            }
            const uint32_t idx = (e >> 5) & 0x3ffff;
            const int m = n - L1;  // <= L2
            const uint32_t rest = code & ((1u << m) - 1);
            const uint32_t lo = rest << (L2 - m), hi = (rest + 1) << (L2 - m);
            for (uint32_t v = lo; v < hi; v++) l2[idx * 128 + v] = pack(m, run, lv, kind);
        }
    }
}

static Tables* build_tables() {
    Tables* t = new Tables();
    t->mba.init(11);
    add_list(t->mba, kMbaCodes);
    t->mba.add(kMbaEscape, 100);
    t->mbtype[1].init(6);
    add_list(t->mbtype[1], kMbTypeI);
    t->mbtype[2].init(6);
    add_list(t->mbtype[2], kMbTypeP);
    t->mbtype[3].init(6);
    add_list(t->mbtype[3], kMbTypeB);
    t->cbp.init(9);
    add_list(t->cbp, kCbpCodes);
    t->motion.init(10);
    add_list(t->motion, kMotionCodes);
    t->dc_luma.init(9);
    add_list(t->dc_luma, kDcSizeLuma);
    t->dc_chroma.init(10);
    add_list(t->dc_chroma, kDcSizeChroma);
    for (int tab = 0; tab < 2; tab++) {
        const vlc_code* codes = tab == 0 ? kCoeffZero : kCoeffOne;
        const int n = tab == 0 ? countof(kCoeffZero) : countof(kCoeffOne);
        CoefLut& f = t->coefs[tab];
        f.l1.assign(1u << CoefLut::L1, 0);
        for (int i = 0; i < n; i++) f.add(codes[i].bits, codes[i].a, codes[i].b, CoefLut::NORMAL);
        f.add(tab == 0 ? kCoeffZeroEob : kCoeffOneEob, 0, 0, CoefLut::EOB);
        f.add(kCoeffEscape, 0, 0, CoefLut::ESC);
    }
    return t;
}

const Tables& Tables::get() {
    static Tables* t = build_tables();
    return *t;
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
double trace_phase(const char* name, double t0) {
    static const bool on = getenv("MP2VG_TRACE") != nullptr;
    const double t = now_ms();
    if (on) fprintf(stderr, "[mp2vg] %-24s %9.3f ms\n", name, t - t0);
    return t;
}

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

}  // namespace mp2vg

extern "C" {

int mp2vg_abi_version(void) { return MP2VG_ABI_VERSION; }

const char* mp2vg_last_error(void) { return mp2vg::g_last_error.c_str(); }

const char* mp2vg_status_string(int s) {
    switch (s) {
    case MP2VG_OK: return "ok";
    case MP2VG_E_INVALID: return "invalid argument";
    case MP2VG_E_UNSUPPORTED: return "stream outside the reference's decodable subset";
    case MP2VG_E_HIP: return "HIP runtime error";
    case MP2VG_E_NOMEM: return "out of memory";
    case MP2VG_E_STATE: return "call out of order";
    case MP2VG_E_BITSTREAM: return "bitstream syntax error";
    default: return "unknown status";
    }
}

void mp2vg_free(void* p) { free(p); }

int mp2vg_frame_geometry(const mp2vg_config_t* cfg, int32_t width[3], int32_t height[3],
                         int32_t stride[3], uint64_t* slot_bytes) {
    if (!cfg || cfg->width <= 0 || cfg->height <= 0 || (cfg->width & 15) || (cfg->height & 15) ||
        cfg->chroma_format < 1 || cfg->chroma_format > 3) {
        mp2vg::set_error("bad config geometry");
        return MP2VG_E_INVALID;
    }
    mp2vg::Geom g;
    g.init(cfg->width, cfg->height, cfg->chroma_format);
    for (int i = 0; i < 3; i++) {
        if (width) width[i] = g.pw[i];
        if (height) height[i] = g.ph[i];
        if (stride) stride[i] = g.stride[i];
    }
    if (slot_bytes) *slot_bytes = g.slot_bytes;
    return MP2VG_OK;
}

}  // extern "C"
