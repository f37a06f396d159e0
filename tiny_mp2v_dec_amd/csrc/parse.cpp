// parse.cpp — host record emitter: MPEG-2 elementary stream -> record stream (include/mp2vg.h).
//
// Reproduces the REFERENCE's parse semantics, quirks included, so that the
// records drive the device reconstruct to the reference's exact output:
//   start-code dispatch              decoder.cpp:278-329
//   header parsers                   mp2v_hdr.cpp:4-223, slice header mp2v_hdr.h:345-363
//   W matrices from the QME only     decoder.cpp:154-192
//   slice setup                      decoder.cpp:107-145
//   macroblock parse                 mb_decoder.cpp:341-641 (parse_modes, cbp, MVs, PMV rules,
//                                    skipped MBs, DC prediction, parse_block's VLC loop)
// Where the reference has undefined behaviour the stream is rejected (MP2VG_E_UNSUPPORTED):
// missing QME / partial loads, intra MBs with intra_vlc_format=0, field pictures, dual-prime,
// slices not starting at column 0, skipped MBs in I pictures, MC reads outside the reference
// planes, 4:4:4 with field DCT (reference writes blocks 10/11 outside the MB), concealment MVs in
// P/B pictures, scalable extensions.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <memory>
#include <condition_variable>
#include <mutex>
#include <vector>

#include "syntax.h"

namespace mp2vg {

namespace {

struct PictureHdr {
    int pct = 0;
    int temporal_reference = 0;
    int f_code[2][2] = {{15, 15}, {15, 15}};
    int intra_dc_precision = 0;
    int picture_structure = 3;
    int frame_pred_frame_dct = 1;
    int concealment_motion_vectors = 0;
    int q_scale_type = 0;
    int intra_vlc_format = 0;
    int alternate_scan = 0;
    bool have_pcext = false;
    bool have_qme = false;
    int qme_load[4] = {0, 0, 0, 0};
    uint8_t qme[4][64] = {};
};

struct SliceJob {
    int pic;                  // decode index
    uint64_t byte_off;        // offset of the slice start code
    uint64_t byte_end;        // end of the slice payload (next start code)
};

struct PicWork {
    PictureHdr hdr;
    int fwd = -1, bwd = -1;   // decode indices of reference pictures (L0 / L1)
    int gop = -1;
    // a B picture between the first two anchors of a GOP with closed_gop = 1: it predicts only
    // backward (ISO 13818-2 6.3.8), so its forward reference is not a dependency for sharding
    bool closed_leading_b = false;
    uint8_t W[4][64] = {};
    std::vector<SliceJob> slices;
};

// allocator whose resize() leaves new elements uninitialised (the coefficient array is filled
// completely by the parallel concatenation; zeroing it first would be a serial memset)
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) {}
    template <class U>
    void construct(U* p) {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
};

// A slice's coefficient words: grown without zeroing and written through a raw pointer into a
// per-MB worst-case reservation (a std::vector resize per macroblock was 4 % of the parse)
struct CoefVec {
    uint32_t* d = nullptr;
    size_t n = 0, cap = 0;
    CoefVec() = default;
    CoefVec(const CoefVec&) = delete;
    CoefVec& operator=(const CoefVec&) = delete;
    CoefVec(CoefVec&& o) noexcept : d(o.d), n(o.n), cap(o.cap) { o.d = nullptr, o.n = o.cap = 0; }
    ~CoefVec() { free(d); }
    void swap(CoefVec& o) noexcept { std::swap(d, o.d), std::swap(n, o.n), std::swap(cap, o.cap); }
    uint32_t* data() { return d; }
    const uint32_t* data() const { return d; }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
    // room for at least `need` words (contents kept)
    bool reserve(size_t need) {
        if (need <= cap) return true;
        size_t c = std::max<size_t>(need, 2 * cap);
        uint32_t* nd = (uint32_t*)realloc(d, c * sizeof(uint32_t));
        if (!nd) return false;
        d = nd;
        cap = c;
        return true;
    }
};

struct SliceOut {
    CoefVec coefs;
    int mb_row = -1;
    int status = MP2VG_OK;
    std::string err;
};

struct Ctx {
    const uint8_t* buf;
    uint64_t len;
    Geom g;
    int width, height, mbw, mbh;
    int vertical_size_value = 0;
    std::vector<PicWork> pics;
    mp2vg_stream_headers_t hdrs{};
};

#define FAIL(code, msg)          \
    do {                         \
        out.status = (code);     \
        out.err = (msg);         \
        return;                  \
    } while (0)

// 6-bit reversal: coded_block_pattern bit (5 - i) names block i
static const uint8_t kRev6[64] = {
    0,  32, 16, 48, 8,  40, 24, 56, 4,  36, 20, 52, 12, 44, 28, 60, 2,  34, 18, 50, 10, 42,
    26, 58, 6,  38, 22, 54, 14, 46, 30, 62, 1,  33, 17, 49, 9,  41, 25, 57, 5,  37, 21, 53,
    13, 45, 29, 61, 3,  35, 19, 51, 11, 43, 27, 59, 7,  39, 23, 55, 15, 47, 31, 63};

// One slice -> its MB row of records (mb_decoder.cpp:521-641 for every MB of the slice).
void parse_slice(const Ctx& C, const PicWork& P, const SliceJob& job, mp2vg_mb_t* row_base_all,
                 std::atomic<uint8_t>* row_done, SliceOut& out) {
    const Tables& T = Tables::get();
    const PictureHdr& h = P.hdr;
    const int pct = h.pct;
    const int cf = C.g.cf;
    const int nblocks = C.g.nblocks;
    // the reader continues past the slice into the bytes after it, as the reference's does
    BitReader br(C.buf + job.byte_off, C.buf + job.byte_end, C.buf + C.len);
    if (!out.coefs.reserve(4096)) FAIL(MP2VG_E_NOMEM, "out of host memory");

    // slice header (mp2v_hdr.h:345-363)
    br.skip(24);
    int vpos = (int)br.read(8);
    int mb_row;
    if (C.vertical_size_value > 2800) {
        int ext = (int)br.read(3);
        mb_row = (ext << 7) + vpos - 1;
    } else {
        mb_row = vpos - 1;
    }
    int qcode = (int)br.read(5);
    if (br.peek(1) == 1) {
        br.skip(1 + 1 + 1 + 6);
        while (br.peek(1) == 1) br.skip(9);
    }
    br.skip(1);
    if (mb_row < 0 || mb_row >= C.mbh) FAIL(MP2VG_E_UNSUPPORTED, "slice row outside the picture");
    // slices of one picture run on several workers: the row is claimed atomically
    if (row_done[mb_row].exchange(1, std::memory_order_relaxed)) FAIL(MP2VG_E_UNSUPPORTED, "two slices in one macroblock row");
    out.mb_row = mb_row;

    // cache setup (decoder.cpp:125-145)
    int16_t PMVs[2][2][2] = {};
    uint16_t dc_pred[3];
    const uint16_t dc_reset = (uint16_t)(1 << (h.intra_dc_precision + 7));
    dc_pred[0] = dc_pred[1] = dc_pred[2] = dc_reset;
    int qscale = qscale_from_code(qcode, h.q_scale_type);
    uint32_t previous_mb_type = 0;
    mp2vg_mb_t* row = row_base_all + (size_t)mb_row * C.mbw;
    int x = 0;
    const int pstruct_frame = 1;  // only frame pictures are accepted
    (void)pstruct_frame;

    auto emit_skipped = [&](int xx) __attribute__((always_inline)) -> bool {
        mp2vg_mb_t& m = row[xx];
        memset(&m, 0, sizeof(m));
        m.x = (uint16_t)xx;
        m.y = (uint16_t)mb_row;
        m.qscale = (uint8_t)qscale;
        m.coef_off = (uint32_t)out.coefs.size();
        // base_motion_compensation<cf, frame, two_vect = (B), skipped=true>(cache, mb, cache.PMVs)
        // (mb_decoder.cpp:546-548, :291-339): direction from previous_mb_type; in B frame
        // pictures vector 1 overwrites vector 0, so the effective vectors are PMVs[1][*].
        uint32_t t = previous_mb_type;
        bool fwd = t & MBT_FWD, bwd = t & MBT_BWD;
        if (!fwd && !bwd) fwd = true;  // 'else' branch: forward
        m.flags = (uint16_t)((fwd ? MP2VG_MB_FWD : 0) | (bwd ? MP2VG_MB_BWD : 0));
        int vsel = (pct == 3) ? 1 : 0;
        for (int s = 0; s < 2; s++)
            for (int c = 0; c < 2; c++) m.mv[0][s][c] = PMVs[vsel][s][c];
        for (int s = 0; s < 2; s++) {
            if (!((s == 0 && fwd) || (s == 1 && bwd))) continue;
            if ((s == 0 ? P.fwd : P.bwd) < 0) return false;
            if (!mc_reads_inside(C.g, xx, mb_row, m.mv[0][s][0], m.mv[0][s][1], false, 0, 0))
                return false;
        }
        return true;
    };

    do {
        if (x >= C.mbw) FAIL(MP2VG_E_BITSTREAM, "macroblock beyond the end of the row");
        // macroblock_address_increment (mb_decoder.cpp:534-539)
        int inc = 0;
        while (br.peek(11) == 0x008) {
            br.skip(11);
            inc += 33;
        }
        int e = T.mba.decode(br);
        if (e < 0 || e >= 33) FAIL(MP2VG_E_BITSTREAM, "bad macroblock_address_increment");
        inc += kMbaCodes[e].a;
        if (x == 0 && inc != 1) FAIL(MP2VG_E_UNSUPPORTED, "slice does not start at column 0");
        // skipped macroblocks (mb_decoder.cpp:541-550)
        if (inc > 1) {
            if (pct == 1) FAIL(MP2VG_E_UNSUPPORTED, "skipped macroblock in an I picture");
            if (pct == 2) memset(PMVs, 0, sizeof(PMVs));
            for (int i = 0; i < inc - 1; i++) {
                if (x >= C.mbw) FAIL(MP2VG_E_BITSTREAM, "skip run beyond the end of the row");
                if (!emit_skipped(x)) FAIL(MP2VG_E_UNSUPPORTED, "skipped MB reads outside the reference");
                x++;
            }
        }
        if (x >= C.mbw) FAIL(MP2VG_E_BITSTREAM, "macroblock beyond the end of the row");

        // macroblock_modes (parse_modes, mb_decoder.cpp:341-419)
        int te = T.mbtype[pct].decode(br);
        if (te < 0) FAIL(MP2VG_E_BITSTREAM, "bad macroblock_type");
        uint32_t mbt = (pct == 1 ? kMbTypeI : pct == 2 ? kMbTypeP : kMbTypeB)[te].a;
        const bool intra = mbt & MBT_INTRA;
        const bool mfwd = mbt & MBT_FWD, mbwd = mbt & MBT_BWD, pattern = mbt & MBT_PATTERN;
        int frame_motion_type = 2;
        if ((mfwd || mbwd) && h.frame_pred_frame_dct == 0) frame_motion_type = (int)br.read(2);
        int dct_type = 0;
        if (h.frame_pred_frame_dct == 0 && (intra || pattern)) dct_type = (int)br.read(1);
        bool field_mv = false;  // mv_format == Field
        int mv_count = 1;
        if (!intra && (mfwd || mbwd)) {
            if (frame_motion_type == 1) {
                field_mv = true;
                mv_count = 2;
            } else if (frame_motion_type == 3) {
                FAIL(MP2VG_E_UNSUPPORTED, "dual-prime prediction");
            } else if (frame_motion_type != 2) {
                FAIL(MP2VG_E_BITSTREAM, "reserved frame_motion_type");
            }
        }
        if (mbt & MBT_QUANT) qscale = qscale_from_code((int)br.read(5), h.q_scale_type);
        if (cf == 3 && dct_type && (intra || pattern))
            FAIL(MP2VG_E_UNSUPPORTED, "4:4:4 field DCT (reference misplaces blocks 10/11)");

        // motion_vectors (mb_decoder.cpp:479-519, 565-574)
        int16_t MVs[2][2][2] = {};
        int fsel[2][2] = {};
        // (always inline: an out-of-line lambda takes br's address and keeps the slice's bit
        // reader in memory, a store-forwarding round trip on every read)
        // one lookup for motion_code and its sign, the residual read with a width of 0 when
        // there is none (f_code 1 or code 0): no branch on the code's value
        auto parse_mv = [&](int r, int s) __attribute__((always_inline)) -> bool {
            for (int t = 0; t < 2; t++) {
                br.refill();  // >= 56 bits: code and sign <= 11, residual <= 8
                const uint32_t e = T.motion_signed[br.peek_nr(11)];
                if (!e) return false;
                br.skip_nr((int)(e >> 16));
                const int mc = (int)(e & 0xffffu) - 32;
                const int fc = h.f_code[s][t];
                const int n = mc != 0 ? fc - 1 : 0;
                const int residual = (int)(((br.cache >> 1) >> (63 - n)) & ((1u << n) - 1u));
                br.skip_nr(n);
                MVs[r][s][t] = mv_reconstruct(fc, mc, residual, PMVs[r][s][t], field_mv && t == 1);
            }
            return true;
        };
        auto parse_mvs = [&](int s) __attribute__((always_inline)) -> bool {
            if (mv_count == 1) {
                if (field_mv) fsel[0][s] = (int)br.read(1);
                return parse_mv(0, s);
            }
            fsel[0][s] = (int)br.read(1);
            if (!parse_mv(0, s)) return false;
            fsel[1][s] = (int)br.read(1);
            return parse_mv(1, s);
        };
        const bool cmv = h.concealment_motion_vectors && pct == 1;
        if (mfwd || (intra && cmv))
            if (!parse_mvs(0)) FAIL(MP2VG_E_BITSTREAM, "bad motion_code");
        if (mbwd)
            if (!parse_mvs(1)) FAIL(MP2VG_E_BITSTREAM, "bad motion_code");
        if (intra && cmv) br.skip(1);

        // PMV update + MC selection (mb_decoder.cpp:580-620)
        mp2vg_mb_t& m = row[x];
        memset(&m, 0, sizeof(m));
        m.x = (uint16_t)x;
        m.y = (uint16_t)mb_row;
        if (pct != 1) {
            bool frame_based = intra || !field_mv;  // prediction_type == Frame_based
            if (frame_based) {
                if (intra) {
                    for (int t = 0; t < 2; t++) PMVs[1][0][t] = PMVs[0][0][t];
                } else if (mfwd && mbwd) {
                    for (int t = 0; t < 2; t++) {
                        PMVs[1][0][t] = PMVs[0][0][t];
                        PMVs[1][1][t] = PMVs[0][1][t];
                    }
                } else if (mfwd) {
                    for (int t = 0; t < 2; t++) PMVs[1][0][t] = PMVs[0][0][t];
                } else if (mbwd) {
                    for (int t = 0; t < 2; t++) PMVs[1][1][t] = PMVs[0][1][t];
                }
            }
            bool no_mc_p = (pct == 2 && !intra && !mfwd);
            if (intra || no_mc_p) {  // concealment is never on in P/B templates
                memset(PMVs, 0, sizeof(PMVs));
                memset(MVs, 0, sizeof(MVs));
                field_mv = false;
            }
            if (!intra) {
                bool fwd = mfwd || no_mc_p, bwd = mbwd;
                m.flags = (uint16_t)((fwd ? MP2VG_MB_FWD : 0) | (bwd ? MP2VG_MB_BWD : 0) |
                                     (field_mv ? MP2VG_MB_FIELD_MC : 0));
                int nv = field_mv ? 2 : 1;
                for (int r = 0; r < nv; r++)
                    for (int s = 0; s < 2; s++) {
                        if (!((s == 0 && fwd) || (s == 1 && bwd))) continue;
                        if ((s == 0 ? P.fwd : P.bwd) < 0)
                            FAIL(MP2VG_E_UNSUPPORTED, "prediction from a missing reference");
                        m.mv[r][s][0] = MVs[r][s][0];
                        m.mv[r][s][1] = MVs[r][s][1];
                        if (field_mv && fsel[r][s]) m.flags |= (uint16_t)MP2VG_MB_FS_BIT(r, s);
                        if (!mc_reads_inside(C.g, x, mb_row, MVs[r][s][0], MVs[r][s][1], field_mv,
                                             fsel[r][s], r))
                            FAIL(MP2VG_E_UNSUPPORTED, "motion vector reads outside the reference");
                    }
            }
        }
        if (intra) m.flags |= MP2VG_MB_INTRA;

        // dct_dc_pred reset (mb_decoder.cpp:623-626)
        if (inc > 1 || !intra) dc_pred[0] = dc_pred[1] = dc_pred[2] = dc_reset;

        // coded_block_pattern (mb_decoder.cpp:421-445, 628-631)
        uint32_t cbp = intra ? 0xfffu : 0;
        if (pattern) {
            int ci = T.cbp.decode(br);
            if (ci < 0) FAIL(MP2VG_E_BITSTREAM, "bad coded_block_pattern");
            uint32_t v = (uint32_t)kCbpCodes[ci].a;
            uint32_t c1 = 0, c2 = 0;
            if (cf == 2) c1 = br.read(2);
            if (cf == 3) c2 = br.read(6);
            // block i <- bit (5 - i) of the code (6.3.17.4), a 6-bit reversal (no branch per bit)
            cbp |= kRev6[v & 63];
            if (cf == 2) cbp |= (uint32_t)(((c1 & 1) << 1) | ((c1 >> 1) & 1)) << 6;
            if (cf == 3) cbp |= (uint32_t)kRev6[c2 & 63] << 6;
        }
        cbp &= (1u << nblocks) - 1;
        if (dct_type && (intra || pattern)) m.flags |= MP2VG_MB_DCT_FIELD;
        m.cbp = (uint16_t)cbp;
        m.qscale = (uint8_t)qscale;
        m.coef_off = (uint32_t)out.coefs.size();

        // blocks (decode_transform_template / decode_block_template / parse_block)
        if (intra && h.intra_vlc_format == 0)
            FAIL(MP2VG_E_UNSUPPORTED, "intra macroblock with intra_vlc_format=0 (reference mis-parses)");
        const int tab = intra ? 1 : 0;
        const CoefLut& cf_lut = T.coefs[tab];
        // room for the MB's worst case (64 words per coded block), written through a raw pointer
        const size_t n0 = out.coefs.size();
        if (!out.coefs.reserve(n0 + 64 * (size_t)__builtin_popcount(cbp))) FAIL(MP2VG_E_NOMEM, "out of host memory");
        uint32_t* w = out.coefs.data() + n0;
        const uint32_t mbx_tag = MP2VG_COEF_MBX(x);
        // the block loop decodes from a local copy of the reader (its address never escapes, so
        // the cache, bit count and pointer stay in registers) and hands it back at the end
        BitReader r = br;
        const uint32_t* const lut1 = cf_lut.l1.data();
        const uint32_t* const lut2 = cf_lut.l2.data();
        // the coded blocks only, lowest first (no data-dependent branch per block position)
        for (uint32_t bits = cbp; bits; bits &= bits - 1) {
            const int b = __builtin_ctz(bits);
            int i = 0;
            const uint32_t btag = ((uint32_t)b << 22) | mbx_tag;  // MP2VG_COEF_PACK's block field
            if (intra) {
                // parse_dct_dc_coeff (mb_decoder.cpp:46-72)
                int pidx = b < 4 ? 0 : ((b & 1) ? 2 : 1);
                int si = (b < 4 ? T.dc_luma : T.dc_chroma).decode(r);  // (refilled: >= 46 bits left)
                if (si < 0) FAIL(MP2VG_E_BITSTREAM, "bad dct_dc_size");
                const int size = (b < 4 ? kDcSizeLuma : kDcSizeChroma)[si].a;  // <= 11
                // dct_dc_differential of `size` bits (none for size 0), without a branch on size
                const int d = (int)(((r.cache >> 1) >> (63 - size)) & ((1u << size) - 1u));
                r.skip_nr(size);
                const int half = (1 << size) >> 1;
                const int diff = d >= half ? d : (d + 1) - 2 * half;
                dc_pred[pidx] = (uint16_t)(dc_pred[pidx] + diff);
                int16_t dcv = (int16_t)(dc_pred[pidx] << (3 - h.intra_dc_precision));
                *w++ = MP2VG_COEF_PACK(dcv, 0, b, MP2VG_COEF_DC | MP2VG_COEF_MBX(x));
                i = 1;
            } else {
                // non-intra first coefficient '1s' (mb_decoder.cpp:79-88), without a branch: the
                // word is stored and kept (w advanced, the two bits consumed) when the bits are '1s'
                const uint32_t c = r.peek(2);
                const uint32_t f = c >> 1;
                *w = MP2VG_COEF_PACK(1 - 2 * (int)(c & 1), 0, b, MP2VG_COEF_FIRST1S | MP2VG_COEF_MBX(x));
                w += f;
                r.skip_nr(2 * (int)f);
                i = (int)f;
            }
            // parse_block's VLC loop (mb_decoder.cpp:89-149): one refill per two codes (a refill
            // leaves >= 56 bits; a code takes at most 24, an escape)
            for (;;) {
                int run, level;
                r.refill();
                int kind = CoefLut::decode_tab(lut1, lut2, r, run, level);
                if (kind != CoefLut::NORMAL) {  // escapes come back as NORMAL (:100-104)
                    if (kind < 0) FAIL(MP2VG_E_BITSTREAM, "bad DCT coefficient code");
                    break;  // EOB
                }
                i += run;
                if (__builtin_expect(i > 63, 0)) FAIL(MP2VG_E_BITSTREAM, "coefficient run past position 63");
                *w++ = ((uint32_t)level & 0xffffu) | ((uint32_t)i << 16) | btag;
                i++;
                kind = CoefLut::decode_tab(lut1, lut2, r, run, level);
                if (kind != CoefLut::NORMAL) {
                    if (kind < 0) FAIL(MP2VG_E_BITSTREAM, "bad DCT coefficient code");
                    break;
                }
                i += run;
                if (__builtin_expect(i > 63, 0)) FAIL(MP2VG_E_BITSTREAM, "coefficient run past position 63");
                *w++ = ((uint32_t)level & 0xffffu) | ((uint32_t)i << 16) | btag;
                i++;
            }
        }
        br = r;
        out.coefs.n = (size_t)(w - out.coefs.data());
        size_t nc = out.coefs.size() - m.coef_off;
        m.ncoef = (uint16_t)nc;
        if (br.overrun()) FAIL(MP2VG_E_BITSTREAM, "slice overruns the buffer");
        previous_mb_type = mbt;
        x++;
    } while (br.peek(23) != 0);
    if (x != C.mbw) FAIL(MP2VG_E_UNSUPPORTED, "slice does not cover the whole macroblock row");
}

#undef FAIL

}  // namespace

struct ParsedImpl {
    std::vector<mp2vg_picture_t> pics;
    std::vector<mp2vg_mb_t, NoInitAlloc<mp2vg_mb_t>> mbs;  // every record is written by its slice
    std::vector<uint32_t, NoInitAlloc<uint32_t>> coefs;
    std::vector<int32_t> display;
    std::vector<int32_t> gop;
    std::vector<int32_t> shard;  // independent decode-order runs (mp2vg_parsed_shards)
    int32_t nshards = 0;
    mp2vg_stream_headers_t hdrs{};
};

}  // namespace mp2vg

struct mp2vg_parsed : mp2vg::ParsedImpl {};

using namespace mp2vg;

// ---- parse session: pass 1 on the caller's thread, pass 2 on worker threads ---------------
// Every slice is a task, as in the reference (decoder.cpp:316-318 queues one task per slice):
// workers claim slices in decode order, so the slices of one picture run on several workers and
// a picture is ready as soon as its last slice is; the worker that finishes it checks its row
// coverage and publishes it (status + its MB records).  mp2vg_parse_es waits for all of them;
// the drop-in decoder consumes pictures as they complete (decoder.cpp), overlapping the parse
// with the device work.
struct ParseSession {
    Ctx C;
    mp2vg_parsed* res = nullptr;  // pictures, MB records (coef_off relative to the slice), display
    std::vector<SliceJob> jobs;
    std::vector<SliceOut> outs;
    std::unique_ptr<std::atomic<uint8_t>[]> row_done;  // picture p's rows at [p * mbh, (p + 1) * mbh)
    std::unique_ptr<std::atomic<int>[]> slices_left;   // per picture
    std::vector<size_t> pic_job_begin;
    std::vector<int> status;  // per picture: 1 pending, else an MP2VG_* status
    std::vector<std::string> err;
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<size_t> next_job{0};
    std::vector<std::thread> workers;
    size_t mbs_per_pic = 0;
    // Streaming (window > 0, the drop-in decoder): a worker parses picture p only once
    // p < consumed + window, into a per-picture MB record buffer that parse_session_append
    // recycles, so host memory stays O(window) for any stream length.  window == 0
    // (mp2vg_parse_es): every picture's records go to res->mbs.
    int window = 0;
    int consumed = 0;  // pictures appended (under mu)
    bool stop = false;  // the consumer is gone: waiting workers return
    std::vector<mp2vg_mb_t*> pic_mbs;  // streaming: picture -> its buffer while parsed, not appended
    std::vector<mp2vg_mb_t*> spare;    // streaming: recycled buffers

    ~ParseSession() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        join();
        for (mp2vg_mb_t* b : pic_mbs) delete[] b;
        for (mp2vg_mb_t* b : spare) delete[] b;
        delete res;
    }
    void join() {
        for (auto& t : workers) t.join();
        workers.clear();
    }
    mp2vg_mb_t* mbs_of(int p) { return window ? pic_mbs[p] : res->mbs.data() + mbs_per_pic * p; }
    void work() {
        for (;;) {
            const size_t j = next_job.fetch_add(1);
            if (j >= jobs.size()) return;
            const int p = jobs[j].pic;
            mp2vg_mb_t* mbs = nullptr;
            if (window) {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || p < consumed + window; });
                if (stop) return;
                if (!pic_mbs[p]) {  // the picture's first slice to get here gives it a buffer
                    if (!spare.empty()) {
                        pic_mbs[p] = spare.back();
                        spare.pop_back();
                    } else {
                        pic_mbs[p] = new mp2vg_mb_t[mbs_per_pic];  // every record is written by its slice
                    }
                }
                mbs = pic_mbs[p];
            } else {
                mbs = mbs_of(p);
            }
            parse_slice(C, C.pics[p], jobs[j], mbs, &row_done[(size_t)p * C.mbh], outs[j]);
            // the last slice of the picture publishes it (acq_rel: every slice's records and
            // outputs are visible to the worker that finishes the picture)
            if (slices_left[p].fetch_sub(1, std::memory_order_acq_rel) == 1) finish_picture(p);
        }
    }
    void finish_picture(int p) {
        int st = MP2VG_OK;
        std::string msg;
        for (size_t j = pic_job_begin[p]; j < pic_job_begin[p + 1]; j++)  // first failing slice in stream order
            if (outs[j].status != MP2VG_OK) {
                char m[256];
                snprintf(m, sizeof m, "picture %d slice @%llu: %s", p, (unsigned long long)jobs[j].byte_off,
                         outs[j].err.c_str());
                st = outs[j].status;
                msg = m;
                break;
            }
        if (st == MP2VG_OK)
            for (int r = 0; r < C.mbh; r++)
                if (!row_done[(size_t)p * C.mbh + r].load(std::memory_order_relaxed)) {
                    st = MP2VG_E_UNSUPPORTED;
                    msg = "picture with a macroblock row not covered by any slice";
                    break;
                }
        {
            std::lock_guard<std::mutex> lk(mu);
            status[p] = st;
            err[p] = msg;
        }
        cv.notify_all();
    }
    int wait(int p) {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return status[p] != 1; });
        if (status[p] != MP2VG_OK) set_error(err[p]);
        return status[p];
    }
};

int parse_session_start(const uint8_t* buf, uint64_t len, const mp2vg_config_t* cfg, int threads, int window,
                        ParseSession** out) {
    if (!buf || !cfg || !out) return MP2VG_E_INVALID;
    *out = nullptr;
    if (mp2vg_frame_geometry(cfg, nullptr, nullptr, nullptr, nullptr) != MP2VG_OK) return MP2VG_E_INVALID;
    std::unique_ptr<ParseSession> S(new ParseSession());
    Ctx& C = S->C;
    C.buf = buf;
    C.len = len;
    C.width = cfg->width;
    C.height = cfg->height;
    C.mbw = cfg->width / 16;
    C.mbh = cfg->height / 16;
    C.g.init(cfg->width, cfg->height, cfg->chroma_format);

    double tp = now_ms();
    // ---- pass 1: start codes and headers, serially (decoder.cpp:278-329) ----
    // start codes 00 00 01 (their 01 byte at k, 2 <= k <= len - 2), found with memchr on 8
    // segments in parallel; each segment owns the 01 bytes inside it
    std::vector<uint64_t> sc;
    {
        const int nseg = len > (1u << 20) ? 8 : 1;
        std::vector<std::vector<uint64_t>> seg(nseg);
        const uint64_t kend = len >= 2 ? len - 1 : 0;  // exclusive bound on k
        parallel_for(nseg, nseg, [&](int j) {
            uint64_t k = std::max<uint64_t>(2, kend * j / nseg);
            const uint64_t hi = kend * (j + 1) / nseg;
            while (k < hi) {
                const void* hit = memchr(buf + k, 1, hi - k);
                if (!hit) break;
                k = (uint64_t)((const uint8_t*)hit - buf);
                if (buf[k - 1] == 0 && buf[k - 2] == 0) seg[j].push_back(k - 2);
                k++;
            }
        });
        for (auto& v : seg) sc.insert(sc.end(), v.begin(), v.end());
    }
    tp = trace_phase("parse: start codes", tp);
    int seq_chroma = -1;
    int cur = -1;
    int gop = -1;
    int ref_frames[2] = {-1, -1};
    bool seq_end = false;
    bool gop_closed = false;
    int gop_anchors = 0;  // anchors decoded since the last group_of_pictures_header
    for (size_t k = 0; k < sc.size() && !seq_end; k++) {
        uint64_t off = sc[k];
        uint64_t end = (k + 1 < sc.size()) ? sc[k + 1] : len;
        uint8_t code = buf[off + 3];
        BitReader br(buf + off, buf + end);
        br.skip(32);
        if (code == 0xB3) {  // sequence_header (mp2v_hdr.cpp:4-21): a later one overwrites
            mp2vg_sequence_header_t& sh = C.hdrs.sequence_header;
            sh.sequence_header_code = 0x1B3;
            sh.horizontal_size_value = br.read(12);
            sh.vertical_size_value = br.read(12);
            sh.aspect_ratio_information = br.read(4);
            sh.frame_rate_code = br.read(4);
            sh.bit_rate_value = br.read(18);
            br.skip(1);  // marker_bit
            sh.vbv_buffer_size_value = br.read(10);
            sh.constrained_parameters_flag = br.read(1);
            sh.load_intra_quantiser_matrix = br.read(1);
            if (sh.load_intra_quantiser_matrix)
                for (int i = 0; i < 64; i++) sh.intra_quantiser_matrix[i] = (uint8_t)br.read(8);
            sh.load_non_intra_quantiser_matrix = br.read(1);
            if (sh.load_non_intra_quantiser_matrix)
                for (int i = 0; i < 64; i++) sh.non_intra_quantiser_matrix[i] = (uint8_t)br.read(8);
            C.vertical_size_value = (int)sh.vertical_size_value;
        } else if (code == 0xB5) {  // extension (decoder.cpp:202-242)
            int id = (int)br.read(4);
            if (id == 1) {  // sequence_extension (mp2v_hdr.cpp:23-37)
                mp2vg_sequence_extension_t& se = C.hdrs.sequence_extension;
                se.extension_start_code_identifier = (uint32_t)id;
                se.profile_and_level_indication = br.read(8);
                se.progressive_sequence = br.read(1);
                se.chroma_format = br.read(2);
                se.horizontal_size_extension = br.read(2);
                se.vertical_size_extension = br.read(2);
                se.bit_rate_extension = br.read(12);
                br.skip(1);  // marker_bit
                se.vbv_buffer_size_extension = br.read(8);
                se.low_delay = br.read(1);
                se.frame_rate_extension_n = br.read(2);
                se.frame_rate_extension_d = br.read(5);
                seq_chroma = (int)se.chroma_format;
            } else if (id == 2) {  // sequence_display_extension (mp2v_hdr.cpp:39-52)
                mp2vg_sequence_display_extension_t& de = C.hdrs.sequence_display_extension;
                de = mp2vg_sequence_display_extension_t{};
                de.extension_start_code_identifier = (uint32_t)id;
                de.video_format = br.read(3);
                de.colour_description = br.read(1);
                if (de.colour_description) {
                    de.colour_primaries = br.read(8);
                    de.transfer_characteristics = br.read(8);
                    de.matrix_coefficients = br.read(8);
                }
                de.display_horizontal_size = br.read(14);
                br.skip(1);  // marker_bit
                de.display_vertical_size = br.read(14);
                C.hdrs.have_sequence_display_extension = 1;
            } else if (id == 5) {
                set_error("scalable extensions are not supported by the reference path");
                return MP2VG_E_UNSUPPORTED;
            } else if (id == 8 && cur >= 0) {  // picture_coding_extension (:105-131)
                PictureHdr& h = C.pics[cur].hdr;
                for (int s = 0; s < 2; s++)
                    for (int t = 0; t < 2; t++) h.f_code[s][t] = (int)br.read(4);
                h.intra_dc_precision = (int)br.read(2);
                h.picture_structure = (int)br.read(2);
                br.skip(1);  // top_field_first
                h.frame_pred_frame_dct = (int)br.read(1);
                h.concealment_motion_vectors = (int)br.read(1);
                h.q_scale_type = (int)br.read(1);
                h.intra_vlc_format = (int)br.read(1);
                h.alternate_scan = (int)br.read(1);
                h.have_pcext = true;
            } else if (id == 3 && cur >= 0) {  // quant_matrix_extension (:133-152)
                PictureHdr& h = C.pics[cur].hdr;
                h.have_qme = true;
                for (int m = 0; m < 4; m++) {
                    h.qme_load[m] = (int)br.read(1);
                    if (h.qme_load[m])
                        for (int i = 0; i < 64; i++) h.qme[m][i] = (uint8_t)br.read(8);
                }
            }
        } else if (code == 0xB8) {  // group_of_pictures_header (mp2v_hdr.cpp:77-83)
            gop++;
            mp2vg_group_of_pictures_header_t& gh = C.hdrs.group_of_pictures_header;
            gh.group_start_code = 0x1B8;
            gh.time_code = br.read(25);
            gh.closed_gop = br.read(1);
            gh.broken_link = br.read(1);
            C.hdrs.have_group_of_pictures_header = 1;
            gop_closed = gh.closed_gop != 0;
            gop_anchors = 0;
        } else if (code == 0x00) {  // picture_start_code (decoder.cpp:294-305)
            PicWork pw;
            pw.hdr.temporal_reference = (int)br.read(10);
            pw.hdr.pct = (int)br.read(3);
            pw.gop = gop < 0 ? 0 : gop;
            if (pw.hdr.pct < 1 || pw.hdr.pct > 3) {
                set_error("unsupported picture_coding_type");
                return MP2VG_E_UNSUPPORTED;
            }
            int idx = (int)C.pics.size();
            if (pw.hdr.pct != 3) {
                pw.fwd = ref_frames[1];  // I/P: dependency on the newest anchor (L0)
                ref_frames[0] = ref_frames[1];
                ref_frames[1] = idx;
                gop_anchors++;
            } else {
                pw.fwd = ref_frames[0];
                pw.bwd = ref_frames[1];
                pw.closed_leading_b = gop_closed && gop_anchors == 1;
            }
            if (pw.hdr.pct == 1) pw.fwd = -1;  // I pictures never predict
            C.pics.push_back(pw);
            cur = idx;
        } else if (code >= 0x01 && code <= 0xAF) {
            if (cur < 0) {
                set_error("slice before the first picture");
                return MP2VG_E_BITSTREAM;
            }
            C.pics[cur].slices.push_back({cur, off, end});
        } else if (code == 0xB7 || code == 0xB4) {
            seq_end = true;
        }
    }
    if (seq_chroma >= 0 && seq_chroma != cfg->chroma_format) {
        set_error("stream chroma_format differs from the decoder configuration");
        return MP2VG_E_UNSUPPORTED;
    }
    // ---- picture-level validation + W (decoder.cpp:154-192) ----
    for (auto& P : C.pics) {
        PictureHdr& h = P.hdr;
        if (!h.have_pcext) { set_error("MPEG-1 picture (no picture_coding_extension)"); return MP2VG_E_UNSUPPORTED; }
        if (h.picture_structure != 3) { set_error("field pictures"); return MP2VG_E_UNSUPPORTED; }
        if (!h.have_qme || !(h.qme_load[0] && h.qme_load[1] && h.qme_load[2] && h.qme_load[3])) {
            set_error("picture without a full quant_matrix_extension (reference decoder.cpp:185-191)");
            return MP2VG_E_UNSUPPORTED;
        }
        if (h.concealment_motion_vectors && h.pct != 1) {
            set_error("concealment motion vectors in a P/B picture");
            return MP2VG_E_UNSUPPORTED;
        }
        if (h.pct == 2 && P.fwd < 0) { set_error("P picture without a reference"); return MP2VG_E_UNSUPPORTED; }
        // f_code of every direction the picture may code vectors for is 1..9 (0 is forbidden and
        // the reference would read f_code - 1 = -1 residual bits, mb_decoder.cpp:500-505)
        for (int s = 0; s < 2; s++) {
            const bool used = (s == 0 && (h.pct != 1 || h.concealment_motion_vectors)) || (s == 1 && h.pct == 3);
            for (int t = 0; t < 2 && used; t++)
                if (h.f_code[s][t] < 1 || h.f_code[s][t] > 9) {
                    set_error("f_code outside 1..9 for a direction the picture codes vectors for");
                    return MP2VG_E_UNSUPPORTED;
                }
        }
        if (P.slices.empty()) { set_error("picture without slices"); return MP2VG_E_BITSTREAM; }
        build_W(h.qme, h.alternate_scan, P.W);
    }
    tp = trace_phase("parse: headers", tp);
    const int npics = (int)C.pics.size();
    const size_t mbs_per_pic = (size_t)C.mbw * C.mbh;
    S->mbs_per_pic = mbs_per_pic;
    auto* res = new mp2vg_parsed();
    S->res = res;
    S->window = std::max(0, window);
    if (S->window)
        S->pic_mbs.assign(npics, nullptr);
    else
        res->mbs.resize(mbs_per_pic * npics);
    for (auto& P : C.pics)
        for (auto& j : P.slices) S->jobs.push_back(j);
    S->outs.resize(S->jobs.size());
    S->row_done.reset(new std::atomic<uint8_t>[(size_t)npics * C.mbh]);
    for (size_t i = 0; i < (size_t)npics * C.mbh; i++) S->row_done[i].store(0, std::memory_order_relaxed);
    S->slices_left.reset(new std::atomic<int>[npics]);
    for (int p = 0; p < npics; p++) S->slices_left[p].store((int)C.pics[p].slices.size(), std::memory_order_relaxed);
    S->pic_job_begin.assign(npics + 1, 0);
    {
        size_t j = 0;
        for (int p = 0; p < npics; p++) {
            S->pic_job_begin[p] = j;
            j += C.pics[p].slices.size();
        }
        S->pic_job_begin[npics] = j;
    }
    S->status.assign(npics, 1);
    S->err.assign(npics, std::string());
    // ---- picture records ----
    res->pics.resize(npics);
    for (int p = 0; p < npics; p++) {
        mp2vg_picture_t& d = res->pics[p];
        memset(&d, 0, sizeof d);
        const PicWork& P = C.pics[p];
        d.dst_slot = p;
        d.fwd_slot = P.fwd;
        d.bwd_slot = P.hdr.pct == 3 ? P.bwd : -1;
        d.picture_coding_type = P.hdr.pct;
        d.mb_first = (uint32_t)(mbs_per_pic * p);
        d.mb_width = (uint16_t)C.mbw;
        d.mb_height = (uint16_t)C.mbh;
        d.alternate_scan = (uint8_t)P.hdr.alternate_scan;
        d.temporal_reference = P.hdr.temporal_reference;
        memcpy(d.W, P.W, sizeof d.W);
        res->gop.push_back(P.gop);
    }
    res->hdrs = C.hdrs;
    // ---- independent shards: a new one starts at p when no picture from p on predicts from a
    // picture before p (references are the two latest anchors, decoder.cpp:299-304) ----
    {
        res->shard.assign(npics, 0);
        int32_t lo = npics;  // min reference of pictures >= p
        std::vector<uint8_t> starts(npics, 0);
        for (int p = npics - 1; p >= 0; p--) {
            const PicWork& P = C.pics[p];
            if (P.fwd >= 0 && !P.closed_leading_b) lo = std::min(lo, (int32_t)P.fwd);
            if (P.hdr.pct == 3 && P.bwd >= 0) lo = std::min(lo, (int32_t)P.bwd);
            starts[p] = lo >= p;
        }
        int32_t sh = -1;
        for (int p = 0; p < npics; p++) {
            if (starts[p] || sh < 0) sh++;
            res->shard[p] = sh;
        }
        res->nshards = sh + 1;
    }
    // ---- display order: the reference's output scheduler (decoder.cpp:346-369) ----
    {
        int held = -1;
        for (int p = 0; p < npics; p++) {
            if (C.pics[p].hdr.pct == 3 || !cfg->reordering) {
                res->display.push_back(p);
            } else {
                if (held >= 0) res->display.push_back(held);
                held = p;
            }
        }
        if (held >= 0) res->display.push_back(held);
    }
    int nthreads = threads > 0 ? threads : cpu_budget();
    nthreads = std::max(1, std::min(nthreads, std::max(1, (int)S->jobs.size())));
    ParseSession* sp = S.get();
    for (int t = 0; t < nthreads; t++) sp->workers.emplace_back([sp]() { sp->work(); });
    *out = S.release();
    return MP2VG_OK;
}

int parse_session_npics(const ParseSession* s) { return (int)s->C.pics.size(); }
const mp2vg_picture_t* parse_session_pictures(const ParseSession* s) { return s->res->pics.data(); }
const int32_t* parse_session_display(const ParseSession* s) { return s->res->display.data(); }
const int32_t* parse_session_shards(const ParseSession* s) { return s->res->shard.data(); }
const mp2vg_stream_headers_t* parse_session_headers(const ParseSession* s) { return &s->res->hdrs; }
int parse_session_wait(ParseSession* s, int p) { return s->wait(p); }
void parse_session_free(ParseSession* s) { delete s; }

// Coefficient words of picture p (after parse_session_wait).
size_t parse_session_ncoefs(const ParseSession* s, int p) {
    size_t n = 0;
    for (size_t j = s->pic_job_begin[p]; j < s->pic_job_begin[p + 1]; j++) n += s->outs[j].coefs.size();
    return n;
}

// Picture p (after parse_session_wait): its MB records into mbs_out and its coefficient words
// into coefs_out, with coef_off relative to coefs_out - base (the picture's words start at word
// `base` of the caller's batch).  The picture's parse buffers are released.
void parse_session_append(ParseSession* s, int p, mp2vg_mb_t* mbs_out, uint32_t* coefs_out, uint32_t base) {
    const size_t n = s->mbs_per_pic;
    memcpy(mbs_out, s->mbs_of(p), n * sizeof(mp2vg_mb_t));
    for (size_t j = s->pic_job_begin[p]; j < s->pic_job_begin[p + 1]; j++) {
        SliceOut& o = s->outs[j];
        if (!o.coefs.empty()) memcpy(coefs_out, o.coefs.data(), o.coefs.size() * 4);
        coefs_out += o.coefs.size();
        mp2vg_mb_t* row = mbs_out + (size_t)o.mb_row * s->C.mbw;
        for (int x = 0; x < s->C.mbw; x++) row[x].coef_off += base;
        base += (uint32_t)o.coefs.size();
        CoefVec().swap(o.coefs);
    }
    if (s->window) {
        {
            std::lock_guard<std::mutex> lk(s->mu);
            s->spare.push_back(s->pic_mbs[p]);
            s->pic_mbs[p] = nullptr;
            s->consumed++;
        }
        s->cv.notify_all();
    }
}

extern "C" int mp2vg_parse_es(const uint8_t* buf, uint64_t len, const mp2vg_config_t* cfg,
                              mp2vg_parsed_t** out) {
    if (!out) return MP2VG_E_INVALID;
    *out = nullptr;
    ParseSession* sp = nullptr;
    int rc = parse_session_start(buf, len, cfg, cfg ? cfg->num_threads : 0, 0, &sp);
    if (rc != MP2VG_OK) return rc;
    std::unique_ptr<ParseSession> S(sp);
    double tp = now_ms();
    S->join();
    const int npics = (int)S->C.pics.size();
    for (int p = 0; p < npics; p++)
        if ((rc = S->wait(p)) != MP2VG_OK) return rc;
    tp = trace_phase("parse: slices", tp);
    // ---- concatenate coefficients, fix offsets: prefix sum, then copies in parallel ----
    std::vector<SliceJob>& jobs = S->jobs;
    std::vector<SliceOut>& outs = S->outs;
    const std::vector<size_t>& pic_job_begin = S->pic_job_begin;
    const size_t mbs_per_pic = S->mbs_per_pic;
    mp2vg_parsed* res = S->res;
    const Ctx& C = S->C;
    std::vector<size_t> base(jobs.size() + 1, 0);
    for (size_t j = 0; j < jobs.size(); j++) base[j + 1] = base[j] + outs[j].coefs.size();
    const size_t total = base[jobs.size()];
    if (total >= (1ull << 32)) {
        set_error("batch too large");
        return MP2VG_E_INVALID;
    }
    res->coefs.resize(total);
    std::atomic<int> next_cp(0);
    auto copier = [&]() {
        for (;;) {
            const int p = next_cp.fetch_add(1);
            if (p >= npics) return;
            for (size_t j = pic_job_begin[p]; j < pic_job_begin[p + 1]; j++) {
                SliceOut& o = outs[j];
                if (!o.coefs.empty()) memcpy(&res->coefs[base[j]], o.coefs.data(), o.coefs.size() * 4);
                mp2vg_mb_t* row = res->mbs.data() + mbs_per_pic * p + (size_t)o.mb_row * C.mbw;
                for (int x = 0; x < C.mbw; x++) row[x].coef_off += (uint32_t)base[j];
                CoefVec().swap(o.coefs);
            }
        }
    };
    int nthreads = cfg->num_threads > 0 ? cfg->num_threads : cpu_budget();
    nthreads = std::max(1, std::min(nthreads, std::max(1, npics)));
    if (nthreads == 1) {
        copier();
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nthreads; t++) th.emplace_back(copier);
        for (auto& t : th) t.join();
    }
    tp = trace_phase("parse: concatenate", tp);
    S->res = nullptr;
    *out = res;
    return MP2VG_OK;
}

extern "C" int mp2vg_parsed_counts(const mp2vg_parsed_t* p, int32_t* npics, uint64_t* nmbs,
                                   uint64_t* ncoefs) {
    if (!p) return MP2VG_E_INVALID;
    if (npics) *npics = (int32_t)p->pics.size();
    if (nmbs) *nmbs = p->mbs.size();
    if (ncoefs) *ncoefs = p->coefs.size();
    return MP2VG_OK;
}
extern "C" const mp2vg_picture_t* mp2vg_parsed_pictures(const mp2vg_parsed_t* p) { return p ? p->pics.data() : nullptr; }
extern "C" const mp2vg_mb_t* mp2vg_parsed_mbs(const mp2vg_parsed_t* p) { return p ? p->mbs.data() : nullptr; }
extern "C" const uint32_t* mp2vg_parsed_coefs(const mp2vg_parsed_t* p) { return p ? p->coefs.data() : nullptr; }
extern "C" int mp2vg_parsed_display_order(const mp2vg_parsed_t* p, int32_t* order, int32_t n) {
    if (!p || !order || n < (int32_t)p->display.size()) return MP2VG_E_INVALID;
    if (!p->display.empty()) memcpy(order, p->display.data(), p->display.size() * 4);
    return (int)p->display.size();
}
extern "C" int mp2vg_parsed_gop_index(const mp2vg_parsed_t* p, int32_t* gop, int32_t n) {
    if (!p || !gop || n < (int32_t)p->gop.size()) return MP2VG_E_INVALID;
    if (!p->gop.empty()) memcpy(gop, p->gop.data(), p->gop.size() * 4);
    return (int)p->gop.size();
}
extern "C" int mp2vg_parsed_stream_headers(const mp2vg_parsed_t* p, mp2vg_stream_headers_t* out) {
    if (!p || !out) return MP2VG_E_INVALID;
    *out = p->hdrs;
    return MP2VG_OK;
}
extern "C" int mp2vg_parsed_shards(const mp2vg_parsed_t* p, int32_t* shard, int32_t n) {
    if (!p || !shard || n < (int32_t)p->shard.size()) return MP2VG_E_INVALID;
    if (!p->shard.empty()) memcpy(shard, p->shard.data(), p->shard.size() * 4);
    return p->nshards;
}
extern "C" void mp2vg_parsed_free(mp2vg_parsed_t* p) { delete p; }
