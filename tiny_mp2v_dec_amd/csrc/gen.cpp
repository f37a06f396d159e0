// gen.cpp — synthetic MPEG-2 elementary-stream writer.
//
// There is no ffmpeg / .m2v corpus here, so golden streams and bench workloads are written by
// this module.  It emits ONLY the subset the reference decodes correctly:
// sequence header + extension, closed GOPs, frame pictures, picture coding extension with
// intra_vlc_format = 1, a full quant_matrix_extension in every picture, one slice per MB row
// starting at column 0 and never ending in a skipped MB, no dual-prime, no skips in I pictures
// or after intra MBs in B pictures, and motion vectors whose reads (half-pel taps included) stay
// inside the reference planes.  The macroblock mix follows SURVEY.md §8d (config C2).
//
// The writer tracks the decoder state exactly as the reference parses it (PMV rules
// mb_decoder.cpp:447-519, 580-604; skipped-MB semantics :541-550; DC prediction :46-72,
// :623-626) so that each chosen motion vector / DC value is what the decoder reconstructs.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#include "syntax.h"

namespace mp2vg {
namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x1234567ull) {}
    uint64_t next() {  // splitmix64
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    int uni(int lo, int hi) { return lo + (int)(next() % (uint64_t)(hi - lo + 1)); }  // inclusive
    bool perm(int permille) { return (int)(next() % 1000) < permille; }
};

struct Enc {
    std::map<std::pair<int, int>, const char*> coef[2];
    Enc() {
        for (int i = 0; i < countof(kCoeffZero); i++) coef[0][{kCoeffZero[i].a, kCoeffZero[i].b}] = kCoeffZero[i].bits;
        for (int i = 0; i < countof(kCoeffOne); i++) coef[1][{kCoeffOne[i].a, kCoeffOne[i].b}] = kCoeffOne[i].bits;
    }
};

const char* find_code(const vlc_code* tab, int n, int a) {
    for (int i = 0; i < n; i++)
        if (tab[i].a == a) return tab[i].bits;
    return nullptr;
}

struct PicParams {
    int pct;
    int tref;
    int alt, qst, prec, fpfd;
    int fcode[2][2];
    bool leading_b;  // backward-only B (closed GOP)
    uint8_t qme[4][64];
};

class Writer {
public:
    Writer(const mp2vg_gen_params_t& p) : P(p), rng(p.seed) {
        g.init(p.width, p.height, p.chroma_format);
        mbw = p.width / 16;
        mbh = p.height / 16;
    }
    int run(std::vector<uint8_t>& out);

private:
    const mp2vg_gen_params_t& P;
    Rng rng;
    Geom g;
    int mbw, mbh;
    BitWriter bw;
    Enc enc;

    // per-slice decoder mirror
    int16_t PMVs[2][2][2];
    uint16_t dc_pred[3];
    uint32_t prev_type;
    int qcode;

    void sequence_header();
    void picture(const PicParams& pp);
    void slice(const PicParams& pp, int row);
    void encode_mv_component(int fcode, int target, int16_t& PMV, bool field_vert);
    void block(const PicParams& pp, bool intra, int b);
    bool choose_vector(int mbx, int mby, bool field, int fs, int s, int16_t out[2]);
    int level_mag();
};

void Writer::sequence_header() {
    bw.start_code(0xB3);
    bw.put(P.width & 0xfff, 12);
    bw.put(P.height & 0xfff, 12);
    bw.put(1, 4);            // aspect_ratio_information
    bw.put(3, 4);            // frame_rate_code (25)
    bw.put(0x3FFFF, 18);     // bit_rate_value
    bw.put(1, 1);            // marker
    bw.put(0x3FF, 10);       // vbv_buffer_size_value
    bw.put(0, 1);            // constrained_parameters_flag
    bw.put(0, 1);            // load_intra_quantiser_matrix (ignored by the reference anyway)
    bw.put(0, 1);            // load_non_intra_quantiser_matrix
    bw.start_code(0xB5);     // sequence_extension
    bw.put(1, 4);
    bw.put(0x44, 8);         // profile_and_level_indication
    bw.put(P.frame_pred_frame_dct ? 1 : 0, 1);  // progressive_sequence
    bw.put(P.chroma_format, 2);
    bw.put(0, 2);
    bw.put(0, 2);
    bw.put(0, 12);
    bw.put(1, 1);
    bw.put(0, 8);
    bw.put(0, 1);            // low_delay
    bw.put(0, 2);
    bw.put(0, 5);
}

int Writer::level_mag() {
    if (rng.perm(P.big_level_permille)) return rng.uni(41, 2047);
    int u = rng.uni(0, 99);
    if (u < 60) return 1;
    if (u < 80) return 2;
    if (u < 90) return 3;
    return rng.uni(4, 40);
}

// motion_code / motion_residual for one component so that the reference's
// update_motion_predictor reconstructs `target` (mb_decoder.cpp:447-477).
void Writer::encode_mv_component(int fcode, int target, int16_t& PMV, bool field_vert) {
    int f = 1 << (fcode - 1);
    int range = 32 * f;
    int pred = field_vert ? (PMV >> 1) : PMV;
    int delta = target - pred;
    while (delta < -16 * f) delta += range;
    while (delta > 16 * f - 1) delta -= range;
    int mc, residual = 0;
    if (f == 1 || delta == 0) {
        mc = delta;
    } else {
        int a = delta < 0 ? -delta : delta;
        mc = (a - 1) / f + 1;
        residual = (a - 1) % f;
        if (delta < 0) mc = -mc;
    }
    int amc = mc < 0 ? -mc : mc;
    bw.put_code(kMotionCodes[amc].bits);
    if (mc) bw.put(mc < 0 ? 1 : 0, 1);
    if (f != 1 && mc != 0) bw.put(residual, fcode - 1);
    int16_t got = mv_reconstruct(fcode, mc, residual, PMV, field_vert);
    if (got != target) {
        fprintf(stderr, "mp2vg gen: MV encode mismatch %d vs %d\n", got, target);
        abort();
    }
}

bool Writer::choose_vector(int mbx, int mby, bool field, int fs, int s, int16_t out[2]) {
    (void)s;
    int f = 1 << (P.f_code - 1);
    for (int tries = 0; tries < 12; tries++) {
        int mx = rng.uni(-16 * f, 16 * f - 1);
        int my = rng.uni(-16 * f, 16 * f - 1);
        if (tries >= 6) {  // shrink towards zero near the picture edges
            mx /= (tries - 4);
            my /= (tries - 4);
        }
        if (mc_reads_inside(g, mbx, mby, mx, my, field, fs, 0)) {
            out[0] = (int16_t)mx;
            out[1] = (int16_t)my;
            return true;
        }
    }
    out[0] = 0;
    out[1] = 0;
    return mc_reads_inside(g, mbx, mby, 0, 0, field, fs, 0);
}

void Writer::block(const PicParams& pp, bool intra, int b) {
    int i = 0;
    if (intra) {
        int pidx = b < 4 ? 0 : ((b & 1) ? 2 : 1);
        int maxv = (1 << (8 + pp.prec)) - 1;
        int target;
        if (rng.perm(150)) target = rng.uni(0, maxv);
        else target = std::min(maxv, std::max(0, (int)dc_pred[pidx] + rng.uni(-24, 24) * (1 << pp.prec)));
        int diff = target - (int)dc_pred[pidx];
        int a = diff < 0 ? -diff : diff;
        int size = 0;
        while ((1 << size) <= a) size++;
        bw.put_code((b < 4 ? kDcSizeLuma : kDcSizeChroma)[size].bits);
        if (size) bw.put(diff > 0 ? diff : diff + (1 << size) - 1, size);
        dc_pred[pidx] = (uint16_t)target;
        i = 1;
    }
    int nmin = intra ? P.intra_coefs_min : std::max(1, P.coefs_min);
    int nmax = intra ? P.intra_coefs_max : std::max(nmin, P.coefs_max);
    int n = rng.uni(nmin, std::max(nmin, nmax));
    int tab = intra ? 1 : 0;
    bool first = !intra;
    int pos = i;
    for (int k = 0; k < n; k++) {
        int run = rng.perm(850) ? rng.uni(0, 3) : rng.uni(0, 20);
        if (pos + run > 63) {
            if (k == 0 && !intra) run = 63 - pos;  // non-intra blocks need one coefficient
            else break;
        }
        int mag = level_mag();
        int sign = (int)(rng.next() & 1);
        bool esc = rng.perm(P.escape_permille);
        if (first && run == 0 && mag == 1 && !esc) {
            bw.put(1, 1);  // '1s' (B.14 first coefficient, mb_decoder.cpp:79-88)
            bw.put(sign, 1);
        } else {
            auto it = enc.coef[tab].find({run, mag});
            if (esc || it == enc.coef[tab].end()) {
                bw.put_code(kCoeffEscape);
                bw.put(run, 6);
                int lv = sign ? -mag : mag;
                bw.put((uint32_t)lv & 0xfff, 12);
            } else {
                bw.put_code(it->second);
                bw.put(sign, 1);
            }
        }
        first = false;
        pos += run + 1;
    }
    bw.put_code(tab ? kCoeffOneEob : kCoeffZeroEob);
}

void Writer::slice(const PicParams& pp, int row) {
    if (P.height > 2800) {
        bw.start_code((uint8_t)((row & 127) + 1));
        bw.put(row >> 7, 3);
    } else {
        bw.start_code((uint8_t)(row + 1));
    }
    qcode = rng.uni(1, 31);
    bw.put(qcode, 5);
    bw.put(0, 1);  // extra_bit_slice
    memset(PMVs, 0, sizeof PMVs);
    uint16_t dc_reset = (uint16_t)(1 << (pp.prec + 7));
    dc_pred[0] = dc_pred[1] = dc_pred[2] = dc_reset;
    prev_type = 0;
    const int pct = pp.pct;
    const int nb = g.nblocks;
    int pending_skip = 0;
    for (int x = 0; x < mbw; x++) {
        // ---- choose the macroblock kind ----
        uint32_t t = 0;
        bool skip = false;
        if (pct == 1 || P.mix == 1) {
            t = MBT_INTRA;
        } else {
            int u = rng.uni(0, 999);
            int intra_pm = P.mix == 2 ? 10 : (pct == 2 ? 100 : 50);
            bool can_skip = x > 0 && x < mbw - 1;
            if (can_skip && pct == 3) {  // B skip: previous coded MB not intra, vectors inside
                if (prev_type & MBT_INTRA) can_skip = false;
                bool fwd = prev_type & MBT_FWD, bwd = prev_type & MBT_BWD;
                if (!fwd && !bwd) can_skip = false;
                if (pp.leading_b && fwd) can_skip = false;
                for (int s = 0; s < 2 && can_skip; s++)
                    if ((s == 0 && fwd) || (s == 1 && bwd))
                        if (!mc_reads_inside(g, x, row, PMVs[1][s][0], PMVs[1][s][1], false, 0, 0)) can_skip = false;
            }
            if (can_skip && u < 100) {
                skip = true;
            } else if (u < 100 + intra_pm) {
                t = MBT_INTRA;
            } else if (pct == 2) {
                int v = rng.uni(0, 99);
                if (v < 67) t = MBT_FWD | MBT_PATTERN;
                else if (v < 73) t = MBT_PATTERN;
                else t = MBT_FWD;
            } else if (pp.leading_b) {
                t = rng.perm(500) ? (MBT_BWD | MBT_PATTERN) : MBT_BWD;
            } else {
                int v = rng.uni(0, 99);
                if (v < 35) t = MBT_FWD | MBT_BWD | MBT_PATTERN;
                else if (v < 53) t = MBT_FWD | MBT_BWD;
                else if (v < 65) t = MBT_BWD | MBT_PATTERN;
                else if (v < 77) t = MBT_BWD;
                else if (v < 89) t = MBT_FWD | MBT_PATTERN;
                else t = MBT_FWD;
            }
        }
        if (skip) {
            pending_skip++;
            continue;
        }
        const bool intra = t & MBT_INTRA;
        if ((intra || (t & MBT_PATTERN)) && rng.perm(P.quant_permille)) t |= MBT_QUANT;
        // ---- macroblock_address_increment ----
        int inc = pending_skip + 1;
        if (inc > 1 && pct == 2) memset(PMVs, 0, sizeof PMVs);  // mb_decoder.cpp:542-543
        while (inc > 33) {
            bw.put_code(kMbaEscape);
            inc -= 33;
        }
        bw.put_code(kMbaCodes[inc - 1].bits);
        // ---- macroblock_type ----
        const vlc_code* tab = pct == 1 ? kMbTypeI : (pct == 2 ? kMbTypeP : kMbTypeB);
        int ntab = pct == 1 ? countof(kMbTypeI) : (pct == 2 ? countof(kMbTypeP) : countof(kMbTypeB));
        const char* code = find_code(tab, ntab, (int)t);
        if (!code) {  // no quant variant for this type
            t &= ~MBT_QUANT;
            code = find_code(tab, ntab, (int)t);
        }
        bw.put_code(code);
        const bool fwd = t & MBT_FWD, bwdd = t & MBT_BWD, pattern = t & MBT_PATTERN;
        bool field = false;
        if (fwd || bwdd) {
            if (!P.frame_pred_frame_dct) {
                field = rng.perm(300);
                bw.put(field ? 1 : 2, 2);  // frame_motion_type
            }
        }
        int dct_type = 0;
        if (!P.frame_pred_frame_dct && (intra || pattern)) {
            dct_type = (g.cf != 3) ? (int)(rng.next() & 1) : 0;
            bw.put(dct_type, 1);
        }
        if (t & MBT_QUANT) {
            qcode = rng.uni(1, 31);
            bw.put(qcode, 5);
        }
        // ---- motion vectors ----
        for (int s = 0; s < 2; s++) {
            if (!((s == 0 && fwd) || (s == 1 && bwdd))) continue;
            if (!field) {
                int16_t v[2];
                choose_vector(x, row, false, 0, s, v);
                for (int c = 0; c < 2; c++) encode_mv_component(pp.fcode[s][c], v[c], PMVs[0][s][c], false);
            } else {
                for (int r = 0; r < 2; r++) {
                    int fs = (int)(rng.next() & 1);
                    int16_t v[2];
                    if (!choose_vector(x, row, true, fs, s, v)) {
                        fs = r;
                        v[0] = v[1] = 0;
                    }
                    bw.put(fs, 1);
                    for (int c = 0; c < 2; c++)
                        encode_mv_component(pp.fcode[s][c], v[c], PMVs[r][s][c], c == 1);
                }
            }
        }
        // ---- PMV update (mb_decoder.cpp:580-604) ----
        if (pct != 1) {
            bool frame_based = intra || !field;
            if (frame_based) {
                if (intra) {
                    for (int c = 0; c < 2; c++) PMVs[1][0][c] = PMVs[0][0][c];
                } else if (fwd && bwdd) {
                    for (int c = 0; c < 2; c++) {
                        PMVs[1][0][c] = PMVs[0][0][c];
                        PMVs[1][1][c] = PMVs[0][1][c];
                    }
                } else if (fwd) {
                    for (int c = 0; c < 2; c++) PMVs[1][0][c] = PMVs[0][0][c];
                } else if (bwdd) {
                    for (int c = 0; c < 2; c++) PMVs[1][1][c] = PMVs[0][1][c];
                }
            }
            if (intra || (pct == 2 && !fwd)) memset(PMVs, 0, sizeof PMVs);
        }
        if (pending_skip > 0 || !intra) dc_pred[0] = dc_pred[1] = dc_pred[2] = (uint16_t)(1 << (pp.prec + 7));
        // ---- coded_block_pattern ----
        uint32_t cbp = intra ? ((1u << nb) - 1) : 0;
        if (pattern) {
            do {
                cbp = (uint32_t)(rng.next() & ((1u << nb) - 1));
            } while (cbp == 0 || (g.cf == 1 && (cbp & 63) == 0) || (g.cf != 1 && (cbp & 63) == 0 && !rng.perm(300)));
            uint32_t v = 0;
            for (int i = 0; i < 6; i++)
                if (cbp & (1u << i)) v |= 1u << (5 - i);
            bw.put_code(find_code(kCbpCodes, countof(kCbpCodes), (int)v));
            if (g.cf == 2) bw.put(((cbp >> 6) & 1) << 1 | ((cbp >> 7) & 1), 2);
            if (g.cf == 3) {
                uint32_t c2 = 0;
                for (int i = 6; i < 12; i++)
                    if (cbp & (1u << i)) c2 |= 1u << (11 - i);
                bw.put(c2, 6);
            }
        }
        for (int b = 0; b < nb; b++)
            if (cbp & (1u << b)) block(pp, intra, b);
        prev_type = t;
        pending_skip = 0;
    }
}

void Writer::picture(const PicParams& pp) {
    bw.start_code(0x00);
    bw.put(pp.tref & 0x3ff, 10);
    bw.put(pp.pct, 3);
    bw.put(0xFFFF, 16);
    if (pp.pct == 2 || pp.pct == 3) {
        bw.put(0, 1);
        bw.put(7, 3);
    }
    if (pp.pct == 3) {
        bw.put(0, 1);
        bw.put(7, 3);
    }
    bw.put(0, 1);  // extra_bit_picture
    bw.start_code(0xB5);  // picture_coding_extension
    bw.put(8, 4);
    for (int s = 0; s < 2; s++)
        for (int t = 0; t < 2; t++) bw.put(pp.fcode[s][t], 4);
    bw.put(pp.prec, 2);
    bw.put(3, 2);  // frame picture
    bw.put(0, 1);  // top_field_first
    bw.put(pp.fpfd, 1);
    bw.put(0, 1);  // concealment_motion_vectors
    bw.put(pp.qst, 1);
    bw.put(1, 1);  // intra_vlc_format
    bw.put(pp.alt, 1);
    bw.put(0, 1);  // repeat_first_field
    bw.put(pp.fpfd, 1);  // chroma_420_type
    bw.put(pp.fpfd, 1);  // progressive_frame
    bw.put(0, 1);  // composite_display_flag
    bw.start_code(0xB5);  // quant_matrix_extension, all four matrices loaded
    bw.put(3, 4);
    for (int m = 0; m < 4; m++) {
        bw.put(1, 1);
        for (int i = 0; i < 64; i++) bw.put(pp.qme[m][i], 8);
    }
    for (int row = 0; row < mbh; row++) slice(pp, row);
}

int Writer::run(std::vector<uint8_t>& out) {
    sequence_header();
    const int M = std::max(1, P.gop_m);
    const int N = std::max(1, P.gop_n);
    for (int gi = 0; gi < P.n_gops; gi++) {
        bw.start_code(0xB8);
        bw.put(0, 25);
        bw.put(1, 1);  // closed_gop
        bw.put(0, 1);
        // coding order of one closed GOP
        std::vector<PicParams> order;
        auto mk = [&](int pct, int tref, bool leading) {
            PicParams pp;
            memset(&pp, 0, sizeof pp);
            pp.pct = (P.mix == 1) ? 1 : pct;
            pp.tref = tref;
            pp.alt = P.alternate_scan >= 0 ? P.alternate_scan : (int)(rng.next() & 1);
            pp.qst = P.q_scale_type >= 0 ? P.q_scale_type : (int)(rng.next() & 1);
            pp.prec = P.intra_dc_precision >= 0 ? P.intra_dc_precision : rng.uni(0, 3);
            pp.fpfd = P.frame_pred_frame_dct;
            for (int s = 0; s < 2; s++)
                for (int t = 0; t < 2; t++) pp.fcode[s][t] = 15;
            if (pp.pct >= 2) pp.fcode[0][0] = pp.fcode[0][1] = P.f_code;
            if (pp.pct == 3) pp.fcode[1][0] = pp.fcode[1][1] = P.f_code;
            pp.leading_b = leading;
            for (int m = 0; m < 4; m++)
                for (int i = 0; i < 64; i++) {
                    int v = rng.perm(P.big_matrix_permille) ? rng.uni(129, 255) : rng.uni(8, 40);
                    pp.qme[m][i] = (uint8_t)v;
                }
            order.push_back(pp);
        };
        int lead = (P.leading_b && M > 1) ? M - 1 : 0;
        mk(1, lead, false);
        for (int k = 0; k < lead; k++) mk(3, k, true);
        int disp = lead + 1;
        while (disp + M - 1 < N + (lead ? 0 : 0) && disp + M - 1 <= N - 1) {
            int ptref = disp + M - 1;
            mk(2, ptref, false);
            for (int k = 0; k < M - 1; k++) mk(3, disp + k, false);
            disp += M;
        }
        for (auto& pp : order) picture(pp);
    }
    bw.start_code(0xB7);  // sequence_end_code
    out.swap(bw.out);
    return 0;
}

}  // namespace
}  // namespace mp2vg

extern "C" void mp2vg_gen_default_params(mp2vg_gen_params_t* p) {
    memset(p, 0, sizeof *p);
    p->width = 352;
    p->height = 288;
    p->chroma_format = 1;
    p->n_gops = 1;
    p->gop_n = 12;
    p->gop_m = 3;
    p->seed = 1729;
    p->frame_pred_frame_dct = 1;
    p->alternate_scan = -1;
    p->q_scale_type = -1;
    p->intra_dc_precision = -1;
    p->coefs_min = 1;
    p->coefs_max = 8;
    p->intra_coefs_min = 0;
    p->intra_coefs_max = 12;
    p->big_level_permille = 5;
    p->escape_permille = 20;
    p->quant_permille = 50;
    p->f_code = 2;
    p->mix = 0;
    p->leading_b = 1;
    p->big_matrix_permille = 0;
}

extern "C" int mp2vg_generate_es(const mp2vg_gen_params_t* p, uint8_t** out, uint64_t* len) {
    if (!p || !out || !len || p->width <= 0 || p->height <= 0 || (p->width & 15) || (p->height & 15) ||
        p->chroma_format < 1 || p->chroma_format > 3 || p->f_code < 1 || p->f_code > 9 ||
        p->width > 4095 || p->height > 4095 || p->n_gops < 1)
        return MP2VG_E_INVALID;
    std::vector<uint8_t> buf;
    mp2vg::Writer w(*p);
    w.run(buf);
    // 64 zero bytes of slack: the reference's scanner / bit reader read past the end
    *len = buf.size();
    uint8_t* m = (uint8_t*)malloc(buf.size() + 64);
    if (!m) return MP2VG_E_NOMEM;
    memcpy(m, buf.data(), buf.size());
    memset(m + buf.size(), 0, 64);
    *out = m;
    return MP2VG_OK;
}
