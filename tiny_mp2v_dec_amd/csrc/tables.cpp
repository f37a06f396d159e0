#include <pthread.h>
#include <sched.h>

#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
// tables.cpp — decode LUTs built once from the Annex B code lists in vlc_tables.h, scan tables,
// error plumbing shared by the whole library.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

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
            // an escape's entry counts its 18 bits of run and level too (decode_entry skips the
            // entry's length alone: no add on the code-to-code dependency chain)
            for (uint32_t v = lo; v < hi; v++) l1[v] = pack(kind == ESC ? n + 18 : n, run, lv, kind);
        } else {
            const uint32_t pre = code >> (n - L1);
            uint32_t& e = l1[pre];
            if (((e >> 23) & 3) != SUB) {
                const uint32_t idx = (uint32_t)(l2.size() >> L2);
                l2.resize(l2.size() + (1u << L2), 0);
                e = pack(0, 0, 0, SUB) | (idx << 5);
            }
            const uint32_t idx = (e >> 5) & 0x3ffff;
            const int m = n - L1;  // <= L2
            const uint32_t rest = code & ((1u << m) - 1);
            const uint32_t lo = rest << (L2 - m), hi = (rest + 1) << (L2 - m);
            for (uint32_t v = lo; v < hi; v++) l2[(idx << L2) + v] = pack(m, run, lv, kind);
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
    t->motion_signed.assign(1u << 11, 0);
    for (const vlc_code& m : kMotionCodes) {
        const int len = (int)strlen(m.bits);
        uint32_t code = 0;
        for (int i = 0; i < len; i++) code = (code << 1) | (m.bits[i] == '1');
        for (int sign = 0; sign < (m.a ? 2 : 1); sign++) {
            const int n = m.a ? len + 1 : len;
            const uint32_t c = m.a ? (code << 1) | (uint32_t)sign : code;
            const int v = sign ? -m.a : m.a;
            for (uint32_t x = c << (11 - n); x < (c + 1) << (11 - n); x++)
                t->motion_signed[x] = ((uint32_t)n << 16) | (uint32_t)(v + 32);
        }
    }
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

// Persistent helper threads for short data-parallel host steps (batch validation, the drop-in
// decoder's record gather, the start-code scan).  Spawning threads per call cost about 0.6 ms per
// 16-picture batch.  One job at a time; the caller works on the job too.
namespace {
class HelperPool {
  public:
    explicit HelperPool(int n) {
        for (int i = 0; i < n; i++) th_.emplace_back([this] { loop(); });
    }
    ~HelperPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return (int)th_.size(); }
    void pin(const cpu_set_t& set) {
        for (auto& t : th_) pthread_setaffinity_np(t.native_handle(), sizeof(set), &set);
    }
    void run(int n, int helpers, const std::function<void(int)>& fn) {
        std::lock_guard<std::mutex> call(call_mu_);
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            n_ = n;
            next_.store(0);
            slots_ = helpers;
            gen_++;
        }
        cv_.notify_all();
        for (int i; (i = next_.fetch_add(1)) < n;) fn(i);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return running_ == 0; });
        fn_ = nullptr;
        slots_ = 0;
    }

  private:
    void loop() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            // join only while indices are left: the caller stops waiting once running_ is 0 after
            // its own loop has claimed the last index
            if (slots_ <= 0 || !fn_ || next_.load() >= n_) continue;
            slots_--;
            running_++;
            const std::function<void(int)>* fn = fn_;
            const int n = n_;
            lk.unlock();
            for (int i; (i = next_.fetch_add(1)) < n;) (*fn)(i);
            lk.lock();
            if (--running_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    int n_ = 0, slots_ = 0, running_ = 0;
    std::atomic<int> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};
}  // namespace

int cpu_budget() {
    static const int budget = [] {
        int n = (int)std::thread::hardware_concurrency();
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::min(n, std::max(1, CPU_COUNT(&set)));
        if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = {0};
            long long period = 0;
            if (fscanf(f, "%31s %lld", q, &period) == 2 && period > 0 && q[0] >= '0' && q[0] <= '9')
                n = std::min(n, (int)std::max(1LL, atoll(q) / period));
            fclose(f);
        }
        return std::max(1, n);
    }();
    return budget;
}

static HelperPool* helper_pool() {
    static HelperPool* pool = new HelperPool(std::max(0, std::min(15, cpu_budget() - 1)));  // never destroyed
    return pool;
}

void parallel_for_pin(const cpu_set_t& set) { helper_pool()->pin(set); }

bool device_local_cpus(const char* pci_bus_id, cpu_set_t* out) {
    std::string id(pci_bus_id);
    for (auto& ch : id) ch = (char)tolower((unsigned char)ch);
    FILE* f = fopen(("/sys/bus/pci/devices/" + id + "/local_cpulist").c_str(), "r");
    if (!f) return false;
    char buf[4096] = {0};
    const bool got = fgets(buf, sizeof(buf), f) != nullptr;
    fclose(f);
    if (!got) return false;
    cpu_set_t allowed, set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return false;
    for (char* p = buf; *p && *p != '\n';) {  // "0-63,128-191"
        char* e;
        long a = strtol(p, &e, 10), b = a;
        if (e == p) break;
        if (*e == '-') b = strtol(e + 1, &e, 10);
        for (long c = a; c <= b && c < CPU_SETSIZE; c++)
            if (c >= 0 && CPU_ISSET(c, &allowed)) CPU_SET(c, &set);
        p = *e == ',' ? e + 1 : e;
    }
    if (CPU_COUNT(&set) == 0) return false;
    *out = set;
    return true;
}

void parallel_for(int n, int max_threads, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    HelperPool* pool = helper_pool();
    const int helpers = std::min({max_threads - 1, pool->size(), n - 1});
    if (helpers <= 0) {
        for (int i = 0; i < n; i++) fn(i);
        return;
    }
    pool->run(n, helpers, fn);
}

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

}  // namespace mp2vg

extern "C" {

int mp2vg_abi_version(void) { return MP2VG_ABI_VERSION; }

int mp2vg_cpu_budget(void) { return mp2vg::cpu_budget(); }

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

// Conformance hook: one code through the host emitter's own Annex B decoders (the LUTs parse.cpp
// uses), for the per-entry VLC tests against the reference's decoders (tests/test_vlc.py).
int mp2vg_vlc_decode(int32_t table, uint64_t bits, int32_t* value, int32_t* aux, int32_t* consumed) {
    using namespace mp2vg;
    if (!value || !aux || !consumed) return MP2VG_E_INVALID;
    uint8_t buf[16] = {};
    for (int i = 0; i < 8; i++) buf[i] = (uint8_t)(bits >> (56 - 8 * i));
    BitReader br(buf, buf + sizeof buf);
    const Tables& T = Tables::get();
    *aux = 0;
    int idx = -1;
    switch (table) {
    case MP2VG_VLC_MBA:
        idx = T.mba.decode(br);
        *value = idx == 100 ? -33 : (idx >= 0 ? kMbaCodes[idx].a : 0);  // escape: +33 to the next code
        break;
    case MP2VG_VLC_MBTYPE_I:
    case MP2VG_VLC_MBTYPE_P:
    case MP2VG_VLC_MBTYPE_B: {
        const int pct = table - MP2VG_VLC_MBTYPE_I + 1;
        idx = T.mbtype[pct].decode(br);
        if (idx >= 0) *value = (int32_t)(pct == 1 ? kMbTypeI : pct == 2 ? kMbTypeP : kMbTypeB)[idx].a;
        break;
    }
    case MP2VG_VLC_CBP:
        idx = T.cbp.decode(br);
        if (idx >= 0) *value = kCbpCodes[idx].a;
        break;
    case MP2VG_VLC_MOTION:  // magnitude, then the sign bit of a non-zero code (mb_decoder.cpp:479-519)
        idx = T.motion.decode(br);
        if (idx >= 0) {
            int mc = kMotionCodes[idx].a;
            if (mc && br.read(1)) mc = -mc;
            *value = mc;
        }
        break;
    case MP2VG_VLC_DC_LUMA:
    case MP2VG_VLC_DC_CHROMA:
        idx = (table == MP2VG_VLC_DC_LUMA ? T.dc_luma : T.dc_chroma).decode(br);
        if (idx >= 0) *value = (table == MP2VG_VLC_DC_LUMA ? kDcSizeLuma : kDcSizeChroma)[idx].a;
        break;
    case MP2VG_VLC_COEF_B14:
    case MP2VG_VLC_COEF_B15: {  // run, signed level (sign bit / escape fields consumed); EOB: run -1
        int run = 0, level = 0;
        const int kind = T.coefs[table - MP2VG_VLC_COEF_B14].decode(br, run, level);
        idx = kind < 0 ? -1 : 0;
        *value = kind == CoefLut::EOB ? -1 : run;
        *aux = level;
        break;
    }
    default:
        set_error("mp2vg_vlc_decode: no decoder for this table (dual-prime dmvector is unsupported)");
        return MP2VG_E_UNSUPPORTED;
    }
    *consumed = (int32_t)br.bitpos();
    if (idx < 0) {
        set_error("mp2vg_vlc_decode: invalid code");
        return MP2VG_E_BITSTREAM;
    }
    return MP2VG_OK;
}

}  // extern "C"
