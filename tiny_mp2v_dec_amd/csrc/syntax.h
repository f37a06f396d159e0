// syntax.h — host-side MPEG-2 syntax helpers shared by the record emitter (parse.cpp) and the
// synthetic stream writer (gen.cpp): bit reader/writer, VLC LUTs, and the small pieces of the
// reference's parse semantics both must agree on (qscale mapping, MV prediction, W build, MC
// read extents).
#pragma once
#include <sched.h>
#include <cstdint>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../include/mp2vg.h"
#include "vlc_tables.h"

namespace mp2vg {

// ---------------------------------------------------------------------------------------------
// MSB-first bit reader over a byte buffer.  Plays the role of the reference's
// bitstream_reader_c (bitstream.h:22-64), which also reads on past a slice's end into the bytes
// that follow it; peek(n) for n <= 32.  The bits are those of [b, hard_end), then zeros; `end`
// (<= hard_end) is the unit being parsed (a slice), which overrun() checks against.
struct BitReader {
    const uint8_t* base = nullptr;
    const uint8_t* p = nullptr;
    const uint8_t* end = nullptr;
    const uint8_t* hend = nullptr;  // bytes at or past hend read as 0
    const uint8_t* lim = nullptr;   // last p with an 8-byte load inside [base, hend)
    uint64_t cache = 0;
    int bits = 0;  // valid bits in cache (MSB aligned); the bits below them are the stream's next

    BitReader() = default;
    BitReader(const uint8_t* b, const uint8_t* e) : BitReader(b, e, e) {}
    BitReader(const uint8_t* b, const uint8_t* e, const uint8_t* hard_end)
        : base(b), p(b), end(e), hend(hard_end), lim(hard_end - b >= 8 ? hard_end - 8 : nullptr) {}

    // Leaves 56-63 valid bits.  Branch-free fast path (no test on `bits`, whose pattern is
    // unpredictable): one unaligned 8-byte big-endian load ORed in below the valid bits, p
    // advanced by the whole bytes that fit.  The bits it leaves below the valid ones are the
    // stream's next bits, so ORing them again later changes nothing.
    inline void refill() {
        if (__builtin_expect(p <= lim, 1)) {
            uint64_t v;
            memcpy(&v, p, 8);
            cache |= __builtin_bswap64(v) >> bits;
            p += (63 - bits) >> 3;
            bits |= 56;
            return;
        }
        refill_tail();
    }
    // (inline: an out-of-line call would take the reader's address and pin a hot loop's local
    // reader to the stack)
    inline void refill_tail() {
        while (bits <= 56) {
            uint64_t byte = (p < hend) ? *p : 0;
            cache |= byte << (56 - bits);
            p++;
            bits += 8;
        }
    }
    inline uint32_t peek(int n) {  // n <= 32
        if (n == 0) return 0;
        refill();
        return (uint32_t)(cache >> (64 - n));
    }
    inline void skip(int n) {
        if (__builtin_expect(n > 32, 0)) return skip_long(n);
        refill();
        cache <<= n;
        bits -= n;
    }
    __attribute__((noinline)) void skip_long(int n) {
        while (n > 32) {
            refill();
            cache <<= 32;
            bits -= 32;
            n -= 32;
        }
        refill();
        cache <<= n;
        bits -= n;
    }
    inline uint32_t read(int n) {  // n <= 32: one refill covers the peek and the skip
        if (n == 0) return 0;
        refill();
        const uint32_t v = (uint32_t)(cache >> (64 - n));
        cache <<= n;
        bits -= n;
        return v;
    }
    // No-refill variants for a caller that has just refilled (>= 33 valid bits) and consumes at
    // most that many before the next refill: the DCT coefficient loop does one refill per code.
    inline uint32_t peek_nr(int n) const { return (uint32_t)(cache >> (64 - n)); }  // 1 <= n <= 32
    inline void skip_nr(int n) {
        cache <<= n;
        bits -= n;
    }
    uint64_t bitpos() const { return (uint64_t)(p - base) * 8 - bits; }
    bool overrun() const { return p > end + 8; }
};

// MSB-first bit writer
struct BitWriter {
    std::vector<uint8_t> out;
    uint64_t acc = 0;
    int nacc = 0;

    void put(uint32_t value, int n) {
        for (int i = n - 1; i >= 0; i--) {
            acc = (acc << 1) | ((value >> i) & 1u);
            if (++nacc == 8) {
                out.push_back((uint8_t)acc);
                acc = 0;
                nacc = 0;
            }
        }
    }
    void put_code(const char* bits) {
        for (const char* c = bits; *c; c++) put(*c == '1', 1);
    }
    void align() {  // zero stuffing to the next byte boundary
        while (nacc) put(0, 1);
    }
    void start_code(uint8_t code) {
        align();
        out.push_back(0);
        out.push_back(0);
        out.push_back(1);
        out.push_back(code);
    }
};

// ---------------------------------------------------------------------------------------------
// VLC decode LUT built from a code list: lut[peek(maxlen)] = {len, index}.
struct VlcLut {
    int maxlen = 0;
    std::vector<uint32_t> lut;  // (len << 16) | (index + 1), 0 = invalid

    void add(const char* bits, int index) {
        int len = (int)strlen(bits);
        uint32_t code = 0;
        for (int i = 0; i < len; i++) code = (code << 1) | (bits[i] == '1');
        uint32_t lo = code << (maxlen - len), hi = (code + 1) << (maxlen - len);
        for (uint32_t v = lo; v < hi; v++) lut[v] = ((uint32_t)len << 16) | (uint32_t)(index + 1);
    }
    void init(int ml) {
        maxlen = ml;
        lut.assign(1u << ml, 0);
    }
    // returns index or -1; consumes the code
    inline int decode(BitReader& br) const {  // maxlen <= 32: one refill for the peek and the skip
        br.refill();
        uint32_t e = lut[br.peek_nr(maxlen)];
        if (!e) return -1;
        br.skip_nr((int)(e >> 16));
        return (int)(e & 0xffff) - 1;
    }
};

// DCT coefficient decoder (B.14 / B.15) with the sign bit folded in: one 12-bit lookup decodes
// the common codes completely (sign included); longer codes (up to 16 + sign bits) take a second
// 5-bit lookup.  The escape (6-bit code, 6-bit run, signed 12-bit level) is decoded without a
// branch: it is frequent in noisy content (9 % of the codes of the bench stream) and a branch on
// it mispredicts.
// Entry: bits 0-4 bits consumed (0 = invalid; an escape's 24: code, run and level), 5-10 run,
// 11-22 signed level, 23-24 kind.
struct CoefLut {
    enum { NORMAL = 0, EOB = 1, ESC = 2, SUB = 3, L1 = 12, L2 = 5 };
    std::vector<uint32_t> l1, l2;  // l2: (1 << L2)-entry sub-tables
    static uint32_t pack(int len, int run, int level, int kind) {
        return (uint32_t)len | ((uint32_t)run << 5) | (((uint32_t)level & 0xfff) << 11) | ((uint32_t)kind << 23);
    }
    // code: '0'/'1' string; sign appended for NORMAL codes
    void add(const char* bits, int run, int level, int kind);
    // returns NORMAL (escapes included), EOB or -1; run / level; consumes the code (and the sign
    // bit, or the escape's run and level)
    inline int decode(BitReader& br, int& run, int& level) const {
        br.refill();  // >= 33 bits: the longest code plus the escape's run and level is 24
        return decode_nr(br, run, level);
    }
    // after a refill; consumes at most 24 bits
    inline int decode_nr(BitReader& br, int& run, int& level) const {
        return decode_tab(l1.data(), l2.data(), br, run, level);
    }
    // the same on table pointers held by the caller (a hot loop keeps them, and its local
    // BitReader, in registers)
    static inline int decode_tab(const uint32_t* t1, const uint32_t* t2, BitReader& br, int& run, int& level) {
        uint32_t e = t1[br.peek_nr(L1)];
        if (__builtin_expect(((e >> 23) & 3) == SUB, 0)) {
            br.skip_nr(L1);
            e = t2[(((e >> 5) & 0x3ffff) << L2) + br.peek_nr(L2)];
        }
        const int len = (int)(e & 31);
        if (__builtin_expect(!len, 0)) return -1;
        const int kind = (int)((e >> 23) & 3);
        // escape (6-bit code, then 6-bit run and signed 12-bit level) without a branch: masks
        // select between the entry's (run, level) and the 18 bits after the escape code
        const uint32_t esc = 0u - (uint32_t)(kind == ESC);
        const uint32_t x = (uint32_t)((br.cache << 6) >> 46);
        const uint32_t rl_norm = (e >> 5) & 0x3ffffu;  // run (6 b) | level (12 b) << 6
        const uint32_t rl = (rl_norm & ~esc) | (((x >> 12) | ((x & 0xfffu) << 6)) & esc);
        run = (int)(rl & 63);
        level = (int32_t)(rl << 14) >> 20;  // signed 12 bits
        br.skip_nr(len);  // (an escape's entry length includes its run and level)
        return kind & ~(int)(esc & 2u);  // ESC -> NORMAL
    }
};

struct Tables {
    VlcLut mba, mbtype[4], cbp, motion, dc_luma, dc_chroma;
    // motion_code with its sign folded in (B.10 + the sign bit of a non-zero code), 11-bit index:
    // entry = (bits consumed << 16) | (motion_code + 32), 0 = invalid
    std::vector<uint32_t> motion_signed;
    CoefLut coefs[2];
    static const Tables& get();
};

// ---------------------------------------------------------------------------------------------
// Reference parse semantics shared by emitter and writer.

// quantiser_scale from quantiser_scale_code (decoder.cpp:140-145, mb_decoder.cpp:555-563)
inline int qscale_from_code(int code, int q_scale_type) {
    if (!q_scale_type) return code << 1;
    if (code < 9) return code;
    if (code < 17) return (code - 4) << 1;
    if (code < 25) return (code - 10) << 2;
    return (code - 17) << 3;
}

// update_motion_predictor (mb_decoder.cpp:447-477) for one component.
// field_vert: mv_format == Field && t == 1 in a frame picture.
inline int16_t mv_reconstruct(int f_code, int motion_code, int residual, int16_t& PMV, bool field_vert) {
    int r_size = f_code - 1;
    int f = 1 << r_size;
    int high = 16 * f - 1, low = -16 * f, range = 32 * f;
    // (|code| - 1) * f + residual + 1 with the code's sign, 0 for code 0; f = 1 carries no
    // residual, so the same form gives the code itself (no branch on the code's value)
    const int a = motion_code < 0 ? -motion_code : motion_code;
    const int d = (a - 1) * f + residual + 1;
    int delta = motion_code < 0 ? -d : d;
    delta = motion_code != 0 ? delta : 0;
    int prediction = field_vert ? (PMV >> 1) : PMV;
    int mv = prediction + delta;
    if (mv < low) mv += range;
    if (mv > high) mv -= range;
    int16_t MV = (int16_t)mv;
    PMV = field_vert ? (int16_t)(MV * 2) : MV;
    return MV;
}

// W[k][scan i] from quant_matrix_extension matrices (transmitted in zig-zag order)
// (decoder.cpp:154-192: tmp = raster via g_scan[0]; W = tmp[g_shuffle[alt][i]]).
extern const uint8_t kScanRaster[2][64];  // scan position -> raster index (v*8+u)
inline void build_W(const uint8_t qme[4][64], int alt, uint8_t W[4][64]) {
    uint8_t zz_of_raster[64];
    for (int zz = 0; zz < 64; zz++) zz_of_raster[kScanRaster[0][zz]] = (uint8_t)zz;
    for (int k = 0; k < 4; k++)
        for (int i = 0; i < 64; i++) W[k][i] = qme[k][zz_of_raster[kScanRaster[alt][i]]];
}

// Frame geometry (decoder.cpp:44-68)
struct Geom {
    int cf;
    int pw[3], ph[3], stride[3];
    uint64_t plane_off[3], slot_bytes;
    int mbw_c, mbh_c;  // chroma MB size
    int nblocks;
    void init(int width, int height, int chroma_format) {
        cf = chroma_format;
        stride[0] = (width + 63) & ~63;
        pw[0] = width;
        ph[0] = height;
        if (cf == 3) {
            stride[1] = stride[0];
            pw[1] = width;
            ph[1] = height;
        } else {
            stride[1] = ((stride[0] >> 1) + 63) & ~63;
            pw[1] = width >> 1;
            ph[1] = cf == 1 ? height >> 1 : height;
        }
        stride[2] = stride[1];
        pw[2] = pw[1];
        ph[2] = ph[1];
        plane_off[0] = 0;
        plane_off[1] = (uint64_t)stride[0] * ph[0];
        plane_off[2] = plane_off[1] + (uint64_t)stride[1] * ph[1];
        slot_bytes = plane_off[2] + (uint64_t)stride[2] * ph[2];
        mbw_c = cf == 3 ? 16 : 8;
        mbh_c = cf == 1 ? 8 : 16;
        nblocks = cf == 1 ? 6 : (cf == 2 ? 8 : 12);
    }
};

// Do the reference's MC reads for one vector of one direction stay inside every plane?
// (mb_decoder.cpp:212-289 address arithmetic; SSE2 loads read width(+1 if x half-pel) bytes and
// height(+1 row-step if y half-pel) rows.)
inline bool mc_reads_inside(const Geom& g, int mbx, int mby, int mvx, int mvy, bool field, int fs, int r) {
    for (int plane = 0; plane < 3; plane++) {
        int mx = mvx, my = mvy;
        if (plane > 0) {
            if (g.cf < 3) mx >>= 1;
            if (g.cf < 2) my >>= 1;
        }
        int w = plane == 0 ? 16 : g.mbw_c;
        int h = plane == 0 ? 16 : g.mbh_c;
        int x0 = mbx * w + (mx >> 1);
        int x1 = x0 + w - 1 + (mx & 1);
        int y0, y1;
        if (!field) {
            y0 = mby * h + (my >> 1);
            y1 = y0 + h - 1 + (my & 1);
        } else {
            int hf = h >> 1;
            y0 = mby * h + fs + 2 * (my >> 1);
            y1 = y0 + 2 * (hf - 1) + 2 * (my & 1);
        }
        (void)r;
        if (x0 < 0 || y0 < 0 || x1 > g.pw[plane] - 1 || y1 > g.ph[plane] - 1) return false;
    }
    return true;
}

void set_error(const std::string& msg);

// fn(0) .. fn(n-1) on the calling thread plus up to max_threads - 1 persistent helper threads;
// returns when all calls have returned (tables.cpp)
void parallel_for(int n, int max_threads, const std::function<void(int)>& fn);

// CPUs this process may keep busy: the hardware threads, capped by the affinity mask and by a
// cgroup v2 CPU quota (cpu.max "quota period": a container allowed 16 CPUs' time on a 256-CPU host
// is throttled for the rest of each period once its threads have used it) (tables.cpp)
int cpu_budget();

// The CPUs local to a PCI device (sysfs local_cpulist: its NUMA node) that this process may use;
// false when unknown.  parallel_for_pin restricts the parallel_for helper threads to a set.
bool device_local_cpus(const char* pci_bus_id, cpu_set_t* out);
void parallel_for_pin(const cpu_set_t& set);

// Host phase timing for diagnosis: with MP2VG_TRACE set, trace_phase(name, t0) prints the
// milliseconds since t0 to stderr and returns the current time.
double now_ms();
double trace_phase(const char* name, double t0);

}  // namespace mp2vg

// Streaming parse (parse.cpp): pass 1 (start codes, headers, picture records, display order) on
// the calling thread, pass 2 (slices -> MB records + coefficient words) on `threads` workers that
// publish pictures in about decode order.  mp2vg_parse_es and the drop-in decoder both use it.
struct ParseSession;
// window > 0: parse at most `window` pictures ahead of parse_session_append (bounded host memory)
int parse_session_start(const uint8_t* buf, uint64_t len, const mp2vg_config_t* cfg, int threads, int window,
                        ParseSession** out);
int parse_session_npics(const ParseSession* s);
const mp2vg_picture_t* parse_session_pictures(const ParseSession* s);  // dst_slot = decode index
const int32_t* parse_session_display(const ParseSession* s);           // npics entries
const int32_t* parse_session_shards(const ParseSession* s);            // npics entries (mp2vg_parsed_shards)
const mp2vg_stream_headers_t* parse_session_headers(const ParseSession* s);
int parse_session_wait(ParseSession* s, int p);  // status of picture p once its slices are parsed
size_t parse_session_ncoefs(const ParseSession* s, int p);  // after parse_session_wait
void parse_session_append(ParseSession* s, int p, mp2vg_mb_t* mbs_out, uint32_t* coefs_out, uint32_t base);
void parse_session_free(ParseSession* s);
