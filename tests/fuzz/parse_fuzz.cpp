// Mutation harness for the host record emitter (parse.cpp + tables.cpp), built with
// -fsanitize=address,undefined by tests/test_sanitize.py (the parser consumes
// untrusted bitstreams).  For each input stream: the stream itself must parse; then `iters`
// mutants (bit flips, random byte spans, truncations, span deletions / duplications, start-code
// injections) go through mp2vg_parse_es (2 threads) and through the streaming parse session the
// drop-in decoder uses (window 4, pictures appended in decode order).  A mutant may be rejected
// with any MP2VG_E_* status; it must never read or write out of bounds or hit undefined
// behaviour (the sanitizers abort the run).
// With -DWITH_VALIDATE (linked with runtime.cpp): every mutant that parses, and record batches of
// the unmutated stream with random fields corrupted (flags, cbp, qscale, ncoef, coef_off, vectors,
// slots, picture geometry, coefficient words), also go through mp2vg_batch_validate -- the
// upload's host-side check that guarantees no batch can make the kernel access memory outside
// its buffers -- which must accept or reject each of them cleanly.
//   parse_fuzz <iters> <seed> <stream.m2v> <width> <height> <chroma_format> [...]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "syntax.h"

using namespace mp2vg;

#ifdef WITH_VALIDATE
#include "recon_kernel.h"
// runtime.cpp's kernel launchers live in recon.hip (device code): never reached by validation
namespace mp2vg {
hipError_t launch_recon(int, int, const KArgs&, hipStream_t) { return hipErrorInvalidValue; }
hipError_t launch_tile_convert(const KArgs&, int, const int32_t*, int, int32_t, hipStream_t) { return hipErrorInvalidValue; }
hipError_t launch_digest(const uint64_t*, const int32_t*, int, const uint64_t*, const int32_t*,
                         const int32_t*, const int32_t*, unsigned long long*, hipStream_t) {
    return hipErrorInvalidValue;
}
hipError_t launch_clock_probe(unsigned long long*, int, int, hipStream_t) { return hipErrorInvalidValue; }
hipError_t launch_block_probe(void*, size_t, int, int, void*, hipStream_t) { return hipErrorInvalidValue; }
hipError_t launch_block_random(const void*, size_t, int, int, void*, hipStream_t) { return hipErrorInvalidValue; }
hipError_t launch_pool_scatter(const uint64_t*, int, uint32_t, uint32_t, int, int, int, void*, hipStream_t) {
    return hipErrorInvalidValue;
}
}  // namespace mp2vg
static long g_valid = 0, g_invalid = 0;

// must_pass: the records are the parser's own output, which the drop-in uploads without this
// check (trusted path): the parser must uphold every invariant the validation enforces
static void validate(const mp2vg_config_t& cfg, std::vector<mp2vg_picture_t>& pics, std::vector<mp2vg_mb_t>& mbs,
                     std::vector<uint32_t>& coefs, int32_t nslots, bool must_pass = false) {
    int32_t nl = 0;
    std::vector<int32_t> lop(pics.size() + 1), mode(64);
    const int rc = mp2vg_batch_validate(&cfg, nslots, pics.data(), (int32_t)pics.size(), mbs.data(), mbs.size(),
                                        coefs.data(), coefs.size(), &nl, lop.data(), mode.data(), 64);
    (rc == MP2VG_OK ? g_valid : g_invalid)++;
    if (must_pass && rc != MP2VG_OK) {
        fprintf(stderr, "parser output rejected by the upload validation: %s\n", mp2vg_last_error());
        abort();
    }
}

static void corrupt_and_validate(const mp2vg_config_t& cfg, const mp2vg_parsed_t* p, std::mt19937_64& rng) {
    int32_t n = 0;
    uint64_t nm = 0, nc = 0;
    mp2vg_parsed_counts(p, &n, &nm, &nc);
    if (!n) return;
    std::vector<mp2vg_picture_t> pics(mp2vg_parsed_pictures(p), mp2vg_parsed_pictures(p) + n);
    std::vector<mp2vg_mb_t> mbs(mp2vg_parsed_mbs(p), mp2vg_parsed_mbs(p) + nm);
    std::vector<uint32_t> coefs(mp2vg_parsed_coefs(p), mp2vg_parsed_coefs(p) + nc);
    validate(cfg, pics, mbs, coefs, n, true);
    const int k = 1 + (int)(rng() % 4);
    for (int i = 0; i < k; i++) {
        const int what = (int)(rng() % 10);
        mp2vg_mb_t& m = mbs[rng() % mbs.size()];
        mp2vg_picture_t& P = pics[rng() % pics.size()];
        switch (what) {
        case 0: m.flags ^= (uint16_t)(1u << (rng() % 16)); break;
        case 1: m.cbp = (uint16_t)rng(); break;
        case 2: m.qscale = (uint8_t)rng(); break;
        case 3: m.ncoef = (uint16_t)(m.ncoef + (int)(rng() % 9) - 4); break;
        case 4: m.coef_off = (uint32_t)(m.coef_off + (int)(rng() % 9) - 4); break;
        case 5: m.mv[rng() % 2][rng() % 2][rng() % 2] = (int16_t)rng(); break;
        case 6: (rng() & 1 ? P.fwd_slot : P.bwd_slot) = (int32_t)(rng() % (n + 3)) - 2; break;
        case 7: (rng() & 1 ? P.mb_width : P.mb_height) ^= (uint16_t)(1u << (rng() % 4)); break;
        case 8: m.x ^= (uint16_t)(1u << (rng() % 8)); break;
        default:
            if (!coefs.empty()) coefs[rng() % coefs.size()] ^= 1u << (rng() % 32);
        }
    }
    validate(cfg, pics, mbs, coefs, n + (int32_t)(rng() % 2));
}
#endif

static std::vector<uint8_t> mutate(const std::vector<uint8_t>& in, std::mt19937_64& rng) {
    std::vector<uint8_t> s = in;
    auto pos = [&](size_t n) { return n ? (size_t)(rng() % n) : 0; };
    const int kind = (int)(rng() % 6);
    if (kind == 0) {  // bit flips
        const int n = 1 + (int)(rng() % 8);
        for (int i = 0; i < n && !s.empty(); i++) s[pos(s.size())] ^= (uint8_t)(1u << (rng() % 8));
    } else if (kind == 1) {  // random byte span
        const size_t p = pos(s.size()), n = 1 + rng() % 64;
        for (size_t i = p; i < s.size() && i < p + n; i++) s[i] = (uint8_t)rng();
    } else if (kind == 2) {  // truncation
        s.resize(pos(s.size() + 1));
    } else if (kind == 3) {  // span deletion
        const size_t p = pos(s.size()), n = 1 + rng() % 256;
        s.erase(s.begin() + p, s.begin() + std::min(s.size(), p + n));
    } else if (kind == 4) {  // span duplication
        const size_t p = pos(s.size()), n = std::min<size_t>(1 + rng() % 512, s.size() - p);
        std::vector<uint8_t> span(s.begin() + p, s.begin() + p + n);
        s.insert(s.begin() + pos(s.size() + 1), span.begin(), span.end());
    } else {  // a start code (random code byte) dropped in
        const uint8_t code[4] = {0, 0, 1, (uint8_t)rng()};
        s.insert(s.begin() + pos(s.size() + 1), code, code + 4);
    }
    return s;
}

static int parse_all(const std::vector<uint8_t>& s, const mp2vg_config_t& cfg, std::mt19937_64& rng) {
    mp2vg_parsed_t* p = nullptr;
    const int rc = mp2vg_parse_es(s.data(), s.size(), &cfg, &p);
    (void)rng;
    if (rc == MP2VG_OK) {
#ifdef WITH_VALIDATE
        corrupt_and_validate(cfg, p, rng);
#endif
        int32_t n = 0;
        uint64_t nm = 0, nc = 0;
        mp2vg_parsed_counts(p, &n, &nm, &nc);
        std::vector<int32_t> v(n > 0 ? n : 1);
        mp2vg_parsed_display_order(p, v.data(), n);
        mp2vg_parsed_shards(p, v.data(), n);
        mp2vg_stream_headers_t h;
        mp2vg_parsed_stream_headers(p, &h);
        mp2vg_parsed_free(p);
    }
    return rc;
}

static int parse_streaming(const std::vector<uint8_t>& s, const mp2vg_config_t& cfg) {
    ParseSession* ps = nullptr;
    int rc = parse_session_start(s.data(), s.size(), &cfg, 2, 4, &ps);
    if (rc != MP2VG_OK) return rc;
    const int n = parse_session_npics(ps);
    const size_t mbs = (size_t)(cfg.width / 16) * (cfg.height / 16);
    std::vector<mp2vg_mb_t> m(mbs);
    std::vector<uint32_t> c;
    for (int p = 0; p < n && rc == MP2VG_OK; p++) {
        rc = parse_session_wait(ps, p);
        if (rc != MP2VG_OK) break;
        c.resize(parse_session_ncoefs(ps, p) + 1);
        parse_session_append(ps, p, m.data(), c.data(), 0);
    }
    parse_session_free(ps);  // with workers still ahead when a picture failed
    return rc;
}

int main(int argc, char** argv) {
    if (argc < 7 || (argc - 3) % 4) {
        fprintf(stderr, "usage: %s iters seed stream w h cf [...]\n", argv[0]);
        return 2;
    }
    const int iters = atoi(argv[1]);
    std::mt19937_64 rng(strtoull(argv[2], nullptr, 10));
    long ok = 0, rejected = 0;
    for (int a = 3; a + 3 < argc; a += 4) {
        FILE* f = fopen(argv[a], "rb");
        if (!f) { perror(argv[a]); return 2; }
        std::vector<uint8_t> es;
        for (int ch; (ch = fgetc(f)) != EOF;) es.push_back((uint8_t)ch);
        fclose(f);
        mp2vg_config_t cfg{};
        cfg.width = atoi(argv[a + 1]);
        cfg.height = atoi(argv[a + 2]);
        cfg.chroma_format = atoi(argv[a + 3]);
        cfg.num_threads = 2;
        cfg.reordering = 1;
        if (parse_all(es, cfg, rng) != MP2VG_OK || parse_streaming(es, cfg) != MP2VG_OK) {
            fprintf(stderr, "%s: the unmutated stream failed: %s\n", argv[a], mp2vg_last_error());
            return 1;
        }
        for (int i = 0; i < iters; i++) {
#ifdef WITH_VALIDATE
            parse_all(es, cfg, rng);  // record-level corruption of the unmutated stream
#endif
            const std::vector<uint8_t> s = mutate(es, rng);
            const int r1 = parse_all(s, cfg, rng);
            const int r2 = parse_streaming(s, cfg);
            (r1 == MP2VG_OK ? ok : rejected)++;
            if ((r1 == MP2VG_OK) != (r2 == MP2VG_OK)) {
                fprintf(stderr, "%s mutant %d: whole-stream parse %d, streaming parse %d\n", argv[a], i, r1, r2);
                return 1;
            }
        }
    }
#ifdef WITH_VALIDATE
    printf("{\"mutants_parsed\": %ld, \"mutants_rejected\": %ld, \"batches_valid\": %ld, \"batches_rejected\": %ld}\n",
           ok, rejected, g_valid, g_invalid);
#else
    printf("{\"mutants_parsed\": %ld, \"mutants_rejected\": %ld}\n", ok, rejected);
#endif
    return 0;
}
