// decoder.cpp — drop-in decoder over the record path: the reference's mp2v_decoder_c behaviour
// (decoder.h:82-131) on the GPU.
//
//   decode(buf, len)  (reference decoder.cpp:278-329): parse the whole elementary stream into
//                     records on the host (multi-threaded, parse.cpp), then stream the pictures
//                     through the device in decode-order chunks: each chunk is one record batch
//                     (one launch per dependency level), frames are copied back into host frames
//                     with the reference frame_c layout (stride = round_up(width, 64), planes
//                     Y,U,V; decoder.cpp:44-77) and handed to the renderer.
//   renderer          called on a dedicated render thread, in the reference's display order
//                     (decoder.cpp:346-379: B pictures at once, I/P delayed by one anchor), with
//                     a frame valid only for the duration of the call.
//   decode() returns after every frame has been rendered (reference flush/kill semantics,
//   decoder.cpp:244-254 + threads.cpp:198-211).
#include <pthread.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <cstdlib>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "recon_kernel.h"
#include "syntax.h"

using namespace mp2vg;

namespace mp2vg {
int batch_upload_pinned(mp2vg_ctx_t* c, const mp2vg_picture_t* pics, int32_t npics, const mp2vg_mb_t* mbs,
                        uint64_t nmbs, const uint32_t* coefs, uint64_t ncoefs);
hipStream_t ctx_stream(mp2vg_ctx_t* c);
int ctx_next_bank(const mp2vg_ctx_t* c);
int ctx_wait_upload(mp2vg_ctx_t* c, int bank);
void ctx_set_launch_timing(mp2vg_ctx_t* c, bool on);
}  // namespace mp2vg

namespace {
// pictures per device batch (MP2VG_CHUNK overrides it for measurements)
const int kChunk = getenv("MP2VG_CHUNK") ? std::max(1, atoi(getenv("MP2VG_CHUNK"))) : 16;
// frame download streams (768-frame c2 e2e: 1 stream 6,925-7,124 frames/s, 2: 6,904-6,949, 4:
// 7,451-7,488; MP2VG_DL_STREAMS overrides it for measurements)
constexpr int kMaxDl = 4;
const int kDlStreams = getenv("MP2VG_DL_STREAMS") ? std::min(kMaxDl, std::max(1, atoi(getenv("MP2VG_DL_STREAMS")))) : 4;
// host frames come back by one copy kernel launch per chunk (recon.hip frame_copy_kernel, stores
// over PCIe into the pinned frames) instead of one DMA per frame; MP2VG_DL_KERNEL=0 selects the
// DMA copies (measurements)
const bool kDlKernel = !getenv("MP2VG_DL_KERNEL") || atoi(getenv("MP2VG_DL_KERNEL")) != 0;

// Host frames live in pinned memory, in the device slot layout (= the reference frame_c layout),
// so a decoded slot comes back with one contiguous DMA copy (with MP2VG_DECODER_DEVICE_FRAMES
// they are HBM buffers and the copy is device to device, no PCIe).  They are recycled after the render
// callback returns (a frame is valid only during the callback, reference threads.cpp:75-80).
// The pool belongs to the decoder and is filled when it is created, as the reference allocates
// its picture pool up front (decoder.cpp:381-406).
struct HostFrame {
    uint8_t* data = nullptr;
    mp2vg_frame_t f;
    class FramePool* owner = nullptr;
};

// A frame pool of `cap` frames.  The reference blocks its decoder on a fixed picture pool
// (threads.cpp:164-166 wait_for_render / wait_for_free); here get() blocks while every frame is
// out and the renderer still holds or has queued some (each put() wakes it).  Only when the
// renderer has none -- the frames are all waiting for display order behind a picture that is
// not decoded yet -- does the pool grow past cap, since waiting could never end.
class FramePool {
  public:
    FramePool(size_t bytes, bool device, int dev) : bytes_(bytes), device_(device), dev_(dev) {}
    ~FramePool() {
        if (device_) hipSetDevice(dev_);
        for (HostFrame* f : all_) {
            if (device_)
                hipFree(f->data);
            else
                hipHostFree(f->data);
            delete f;
        }
    }
    bool reserve(int n) {
        cap_ = std::max(cap_, n);
        while ((int)all_.size() < n) {
            HostFrame* f = alloc();
            if (!f) return false;
            put(f);
        }
        return true;
    }
    // renderer_holds(): frames queued for or inside the render callback (under no pool lock)
    HostFrame* get(const std::function<int()>& renderer_holds) {
        {
            std::unique_lock<std::mutex> lk(mu_);
            for (;;) {
                if (!free_.empty()) {
                    HostFrame* f = free_.back();
                    free_.pop_back();
                    return f;
                }
                if ((int)all_.size() < cap_ || renderer_holds() == 0) break;
                cv_.wait_for(lk, std::chrono::milliseconds(20));
            }
        }
        return alloc();
    }
    void put(HostFrame* f) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            free_.push_back(f);
        }
        cv_.notify_all();
    }
    size_t free_count() {
        std::lock_guard<std::mutex> lk(mu_);
        return free_.size();
    }
    size_t size() {
        std::lock_guard<std::mutex> lk(mu_);
        return all_.size();
    }

  private:
    HostFrame* alloc() {
        auto* f = new HostFrame();
        f->owner = this;
        if (device_) hipSetDevice(dev_);
        const hipError_t e = device_ ? hipMalloc((void**)&f->data, bytes_)
                                     : hipHostMalloc((void**)&f->data, bytes_, hipHostMallocDefault);
        if (e != hipSuccess) {
            delete f;
            return nullptr;
        }
        std::lock_guard<std::mutex> lk(mu_);
        all_.push_back(f);
        return f;
    }
    size_t bytes_;
    bool device_;
    int dev_;
    int cap_ = 0;
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<HostFrame*> all_, free_;
};

// Growable pinned host buffer: a chunk's records are gathered here and DMA'd without staging.
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    ~PinnedBuf() {
        if (p) hipHostFree(p);
    }
    bool reserve(size_t bytes) {
        if (bytes <= cap) return true;
        const size_t c = std::max(bytes, cap + cap / 2);
        if (p) hipHostFree(p);
        p = nullptr;
        cap = 0;
        if (hipHostMalloc(&p, c, hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            return false;
        }
        cap = c;
        return true;
    }
};

// One device of the decoder (GOP sharding deals the stream's independent shards to lanes):
// its own record context (frame slots, two record banks, launch streams), download streams,
// and, with MP2VG_DECODER_DEVICE_FRAMES, its own HBM frame pool.
struct Lane {
    int device = 0;
    mp2vg_ctx_t* ctx = nullptr;
    int nslots = 0;
    std::unique_ptr<FramePool> dpool;
    PinnedBuf mbuf[2], cbuf[2];        // chunk MB records / coefficient words, one set per record bank
    // frame downloads, slots dealt round-robin: each stream's copies go to their own DMA engine
    hipStream_t dl[kMaxDl] = {};
    // the host waits for a download stream through one of these (hipEventBlockingSync: the
    // waiting thread sleeps instead of spinning, which on a CPU-quota'd host costs the parse
    // workers their share)
    hipEvent_t dlev[kMaxDl] = {};
    int ndl = 1;
    hipEvent_t decoded = nullptr;      // end of the last chunk's decode (on the context stream)
    int frames = 0;                    // frames decoded in the last decode()
    // per decode() state
    std::vector<int> free_slots;
    std::map<int, HostFrame*> inflight;  // decode index -> frame whose copy is in flight
    std::vector<int> pend;               // pictures of the chunk whose copies are in flight
    uint64_t pend_seq = 0;               // chunk number of `pend` (oldest pending lane first)
    std::vector<int> held;               // copied pictures whose slot a later picture still reads
    ~Lane() {
        hipSetDevice(device);
        for (hipStream_t st : dl)
            if (st) hipStreamSynchronize(st);
        if (ctx) mp2vg_synchronize(ctx);
        dpool.reset();
        if (decoded) hipEventDestroy(decoded);
        for (hipEvent_t e : dlev)
            if (e) hipEventDestroy(e);
        for (hipStream_t st : dl)
            if (st) hipStreamDestroy(st);
        if (ctx) mp2vg_destroy(ctx);
    }
};
}  // namespace

struct mp2vg_decoder {
    mp2vg_config_t cfg{};
    mp2vg_render_fn fn = nullptr;
    void* user = nullptr;
    Geom g{};
    std::vector<std::unique_ptr<Lane>> lanes;
    std::unique_ptr<FramePool> hpool;  // pinned host frames, shared by every lane
    bool device_frames = false;        // MP2VG_DECODER_DEVICE_FRAMES: frames handed over in HBM
    // host frames by the copy kernel: every lane on one device (the pinned pool is mapped for the
    // device it was allocated under; lanes on several devices copy by DMA)
    bool kernel_copy = false;
    mp2vg_stream_headers_t hdrs{};     // of the last decode()
    // the CPUs of the first device's NUMA node (its PCI local_cpulist) that the process may use:
    // with MP2VG_PIN=1 decode()'s threads run there
    bool pin = false;
    cpu_set_t local{};
    // of the last decode(): lane changes that found the lane just left still downloading (its
    // chunk left in flight, the host moving on), and host blocks on another lane's downloads
    // (only when the frame pool runs short); lane changes whose lane just left had nothing in
    // flight or was completed by the non-blocking check; lane changes
    int handoffs_in_flight = 0, handoff_blocks = 0, handoffs_landed = 0, lane_changes = 0;
};

extern "C" int mp2vg_decoder_destroy(mp2vg_decoder_t* d) {
    if (!d) return MP2VG_E_INVALID;
    d->lanes.clear();  // synchronises every lane's streams before its buffers go
    d->hpool.reset();
    delete d;
    return MP2VG_OK;
}

extern "C" int mp2vg_decoder_create_multi(const mp2vg_config_t* cfg, const int32_t* devices, int32_t ndevices,
                                          mp2vg_render_fn fn, void* user, mp2vg_decoder_t** out) {
    if (!cfg || !fn || !out || !devices || ndevices < 1 || ndevices > 64) return MP2VG_E_INVALID;
    *out = nullptr;
    if (cfg->reserved & ~MP2VG_DECODER_DEVICE_FRAMES) {
        set_error("unknown decoder flags in mp2vg_config_t.reserved");
        return MP2VG_E_INVALID;
    }
    auto* d = new mp2vg_decoder();
    d->cfg = *cfg;
    // chunk k decodes into its own slots while chunk k-1 is still being downloaded
    d->cfg.pictures_pool_size = std::max(cfg->pictures_pool_size, 2 * kChunk + 4);
    d->fn = fn;
    d->user = user;
    d->g.init(cfg->width, cfg->height, cfg->chroma_format);
    d->device_frames = cfg->reserved & MP2VG_DECODER_DEVICE_FRAMES;
    // (opt-in, MP2VG_PIN=1: on a shared 2-socket host it did not steady the slow decode() calls,
    // profiles/r6/dropin_pin_ab.txt)
    if (getenv("MP2VG_PIN") && atoi(getenv("MP2VG_PIN"))) {
        char bus[64] = {0};
        d->pin = hipDeviceGetPCIBusId(bus, (int)sizeof(bus), devices[0]) == hipSuccess &&
                 device_local_cpus(bus, &d->local);
    }
    // the copy kernel: into pinned host frames (one device), or into each lane's own HBM frames
    d->kernel_copy = kDlKernel;
    for (int i = 1; i < ndevices; i++) d->kernel_copy = d->kernel_copy && (d->device_frames || devices[i] == devices[0]);
    // frames in flight per lane: one chunk being copied, one being rendered, anchors held for display
    const int frames_per_lane = 2 * kChunk + 4;
    const size_t chunk_mbs = (size_t)kChunk * (cfg->width / 16) * (cfg->height / 16);
    for (int i = 0; i < ndevices; i++) {
        d->lanes.emplace_back(new Lane());
        Lane& L = *d->lanes.back();
        L.device = devices[i];
        mp2vg_config_t c = d->cfg;
        c.device = devices[i];
        c.reserved = 0;
        int rc = mp2vg_create(&c, &L.ctx);
        if (rc != MP2VG_OK) {
            mp2vg_decoder_destroy(d);
            return rc;
        }
        L.nslots = c.pictures_pool_size;
        ctx_set_launch_timing(L.ctx, false);  // no per-launch events on the drop-in's chunk path
        hipSetDevice(L.device);
        L.ndl = kDlStreams;
        bool sok = true;
        for (int k = 0; k < L.ndl; k++)
            sok = sok && hipStreamCreateWithFlags(&L.dl[k], hipStreamNonBlocking) == hipSuccess &&
                  hipEventCreateWithFlags(&L.dlev[k], hipEventBlockingSync | hipEventDisableTiming) == hipSuccess;
        if (!sok || hipEventCreateWithFlags(&L.decoded, hipEventDisableTiming) != hipSuccess) {
            set_error("download stream / event creation failed");
            mp2vg_decoder_destroy(d);
            return MP2VG_E_HIP;
        }
        // chunk record buffers sized up front: every MB record of a chunk, and 32 coefficient
        // words per MB (the bench stream needs 12.5; a chunk that needs more grows its set once)
        bool ok = true;
        for (int k = 0; k < 2; k++)
            ok = ok && L.mbuf[k].reserve(chunk_mbs * sizeof(mp2vg_mb_t)) && L.cbuf[k].reserve(chunk_mbs * 32 * 4);
        if (d->device_frames) {
            L.dpool.reset(new FramePool(d->g.slot_bytes, true, L.device));
            ok = ok && L.dpool->reserve(frames_per_lane);
        }
        if (!ok) {
            set_error("pinned record buffer / device frame allocation failed");
            mp2vg_decoder_destroy(d);
            return MP2VG_E_NOMEM;
        }
    }
    if (!d->device_frames) {
        d->hpool.reset(new FramePool(d->g.slot_bytes, false, devices[0]));
        if (!d->hpool->reserve(frames_per_lane * ndevices)) {
            set_error("pinned host frame allocation failed");
            mp2vg_decoder_destroy(d);
            return MP2VG_E_NOMEM;
        }
    }
    *out = d;
    return MP2VG_OK;
}

extern "C" int mp2vg_decoder_create(const mp2vg_config_t* cfg, mp2vg_render_fn fn, void* user,
                                    mp2vg_decoder_t** out) {
    if (!cfg) return MP2VG_E_INVALID;
    const int32_t dev = cfg->device;
    return mp2vg_decoder_create_multi(cfg, &dev, 1, fn, user, out);
}

extern "C" int mp2vg_decoder_stream_headers(const mp2vg_decoder_t* d, mp2vg_stream_headers_t* out) {
    if (!d || !out) return MP2VG_E_INVALID;
    *out = d->hdrs;
    return MP2VG_OK;
}

extern "C" int mp2vg_decoder_lane_frames(const mp2vg_decoder_t* d, int32_t* frames, int32_t n) {
    if (!d) return MP2VG_E_INVALID;
    for (int i = 0; i < n && i < (int)d->lanes.size(); i++) frames[i] = d->lanes[i]->frames;
    return (int)d->lanes.size();
}

extern "C" int mp2vg_decoder_handoff_stats(const mp2vg_decoder_t* d, int32_t* in_flight, int32_t* blocks,
                                           int32_t* landed, int32_t* changes) {
    if (!d) return MP2VG_E_INVALID;
    if (in_flight) *in_flight = d->handoffs_in_flight;
    if (blocks) *blocks = d->handoff_blocks;
    if (landed) *landed = d->handoffs_landed;
    if (changes) *changes = d->lane_changes;
    return MP2VG_OK;
}

extern "C" int mp2vg_decoder_frames_allocated(const mp2vg_decoder_t* d) {
    if (!d) return MP2VG_E_INVALID;
    size_t n = d->hpool ? d->hpool->size() : 0;
    for (auto& L : d->lanes)
        if (L->dpool) n += L->dpool->size();
    return (int)n;
}

// Runs decode() with the calling thread on the decoder's NUMA-local CPUs: the parse workers and
// the render thread it starts inherit them, the parallel_for helpers are moved there; the caller's
// own affinity comes back on return.
struct LocalCpus {
    bool on = false;
    cpu_set_t saved{};
    explicit LocalCpus(const mp2vg_decoder_t* d) {
        if (!d->pin || pthread_getaffinity_np(pthread_self(), sizeof(saved), &saved) != 0) return;
        on = pthread_setaffinity_np(pthread_self(), sizeof(d->local), &d->local) == 0;
        if (on) parallel_for_pin(d->local);
    }
    ~LocalCpus() {
        if (on) pthread_setaffinity_np(pthread_self(), sizeof(saved), &saved);
    }
};

static int decoder_decode(mp2vg_decoder_t* d, const uint8_t* buf, uint64_t len);

extern "C" int mp2vg_decoder_decode(mp2vg_decoder_t* d, const uint8_t* buf, uint64_t len) {
    if (!d || !buf) return MP2VG_E_INVALID;
    LocalCpus guard(d);
    return decoder_decode(d, buf, len);
}

static int decoder_decode(mp2vg_decoder_t* d, const uint8_t* buf, uint64_t len) {
    // the parse runs on worker threads while the chunks below go through the device: a chunk
    // waits only for its own pictures (one thread is left for this loop; the renderer mostly
    // waits on downloads)
    double t0 = now_ms(), tc;
    double t_up = 0, t_dec = 0, t_down = 0, t_wait = 0, t_gather = 0;
    ParseSession* ps = nullptr;
    const int threads = d->cfg.num_threads > 0 ? d->cfg.num_threads : cpu_budget();
    // Parse workers: the thread budget less three (this feed loop, its gather helpers, the render
    // thread).  On the GPU box's 16-CPU quota (cgroup cpu.max on 256 CPUs) 15 workers of 16 threads
    // left some decode() calls throttled (c2 3,072 frames, device frames: 5.9k next to 9.7-10.3k
    // frames/s), 13 kept every call at 9.8-10.8k (profiles/r6/dropin_threads.jsonl).
    int rc = parse_session_start(buf, len, &d->cfg, std::max(1, threads - 3), 4 * kChunk, &ps);
    t0 = trace_phase("dropin: headers", t0);
    if (rc != MP2VG_OK) return rc;
    std::unique_ptr<ParseSession, void (*)(ParseSession*)> guard(ps, parse_session_free);
    d->hdrs = *parse_session_headers(ps);
    const int32_t npics = parse_session_npics(ps);
    const mp2vg_picture_t* pics = parse_session_pictures(ps);
    std::vector<int32_t> display(parse_session_display(ps), parse_session_display(ps) + npics);
    const int32_t* shard = parse_session_shards(ps);
    const int nl = (int)d->lanes.size();
    // Lanes take runs of whole shards, each run at least a chunk long: consecutive shards merge
    // until the run holds kChunk pictures, and run r goes to lane r % nl.  An I-only stream (one
    // shard per picture) then still feeds each lane full chunks instead of alternating lanes
    // picture by picture (one upload, launch chain and download sync per picture).
    std::vector<int32_t> lane_idx(npics, 0);
    for (int p = 0, run = 0, len = 0; p < npics; p++) {
        if (p > 0 && shard[p] != shard[p - 1] && len >= kChunk) {
            run++;
            len = 0;
        }
        lane_idx[p] = run % nl;
        len++;
    }
    auto lane_of = [&](int p) -> Lane& { return *d->lanes[lane_idx[p]]; };

    // a reference on another lane: the forward anchor of a closed GOP's leading B picture, which
    // its macroblocks never read (mp2vg_parsed_shards); checked on its records below
    auto foreign = [&](int q, int r) { return r >= 0 && &lane_of(r) != &lane_of(q); };
    // last decode index that predicts from each picture (on the picture's own lane)
    std::vector<int> last_use(npics, -1);
    for (int q = 0; q < npics; q++) {
        if (pics[q].fwd_slot >= 0 && !foreign(q, pics[q].fwd_slot)) last_use[pics[q].fwd_slot] = q;
        if (pics[q].bwd_slot >= 0) last_use[pics[q].bwd_slot] = q;
    }

    // render thread (decoder.cpp:403, :346-379)
    std::mutex mu;
    std::condition_variable cv;
    std::deque<HostFrame*> q;
    std::atomic<int> held{0};  // frames queued for or inside the render callback
    bool done = false;
    std::thread render([&]() {
        for (;;) {
            HostFrame* f;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return done || !q.empty(); });
                if (q.empty()) return;
                f = q.front();
                q.pop_front();
            }
            d->fn(d->user, &f->f);
            f->owner->put(f);
            held--;
        }
    });
    auto renderer_holds = [&]() { return held.load(); };

    std::vector<int> slot_of(npics, -1);
    std::vector<uint8_t> queued(npics, 0);  // the picture's decode has been queued
    for (auto& Lp : d->lanes) {
        Lane& L = *Lp;
        L.free_slots.clear();
        for (int s = L.nslots - 1; s >= 0; s--) L.free_slots.push_back(s);
        L.inflight.clear();
        L.pend.clear();
        L.held.clear();
        L.frames = 0;
    }
    std::map<int, HostFrame*> ready;  // decode index -> downloaded frame, waiting for display order
    size_t next_display = 0;
    std::vector<mp2vg_picture_t> cp;
    std::vector<size_t> ncoef_of(kChunk);
    std::vector<uint32_t> base_of(kChunk);
    const uint64_t mbs_per_pic = (uint64_t)(d->cfg.width / 16) * (d->cfg.height / 16);

    auto finish = [&](int status) {
        for (auto& Lp : d->lanes) {  // no copy may still target a pool frame
            hipSetDevice(Lp->device);
            for (int i = 0; i < Lp->ndl; i++) hipStreamSynchronize(Lp->dl[i]);
            mp2vg_synchronize(Lp->ctx);
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            done = true;
        }
        cv.notify_all();
        render.join();
        // frames an error left behind go back to their pools (a long-lived decoder must not grow)
        for (auto& Lp : d->lanes) {
            for (auto& kv : Lp->inflight) kv.second->owner->put(kv.second);
            Lp->inflight.clear();
            Lp->pend.clear();
        }
        for (auto& kv : ready) kv.second->owner->put(kv.second);
        ready.clear();
        return status;
    };

    // Chunk pipeline, per lane; nothing waits for a device except through an event:
    //   host:   gather chunk k's records (pinned) | upload (copy stream; waits only for the decode
    //           of chunk k-2, which read the same record bank) | queue decode k | complete k-1
    //   device: decode k-1 ... decode k (context stream) while the D2H copies of k-1 run (dl)
    // A chunk's frames reach the renderer, and its slots return to the lane's free list, only
    // after its copies have completed; a released slot is rewritten only by a later chunk of the
    // same lane, whose decode is ordered after every earlier one on that lane's context stream.
    auto complete_pending = [&](Lane& L) -> int {
        if (L.pend.empty()) return MP2VG_OK;
        tc = now_ms();
        hipSetDevice(L.device);
        static const bool blocking = !getenv("MP2VG_DL_BLOCKING") || atoi(getenv("MP2VG_DL_BLOCKING"));
        for (int i = 0; i < L.ndl; i++)
            if (blocking ? (hipEventRecord(L.dlev[i], L.dl[i]) != hipSuccess || hipEventSynchronize(L.dlev[i]) != hipSuccess)
                         : hipStreamSynchronize(L.dl[i]) != hipSuccess)
                return MP2VG_E_HIP;
        t_down += now_ms() - tc;
        for (auto& kv : L.inflight) ready[kv.first] = kv.second;
        L.inflight.clear();
        // release this lane's slots that no picture still to be queued predicts from (an anchor
        // stays held until the decode of its last user is queued)
        L.held.insert(L.held.end(), L.pend.begin(), L.pend.end());
        size_t keep = 0;
        for (int p : L.held) {
            if (last_use[p] < 0 || queued[last_use[p]]) {
                L.free_slots.push_back(slot_of[p]);
                slot_of[p] = -1;
            } else {
                L.held[keep++] = p;
            }
        }
        L.held.resize(keep);
        L.pend.clear();
        // hand frames to the render thread in display order
        while (next_display < display.size() && ready.count(display[next_display])) {
            auto it = ready.find(display[next_display]);
            held++;
            {
                std::lock_guard<std::mutex> lk(mu);
                q.push_back(it->second);
            }
            cv.notify_one();
            ready.erase(it);
            next_display++;
        }
        return MP2VG_OK;
    };

    // one chunk: pictures [s, e) in decode order, all of lane L
    auto run_chunk = [&](Lane& L, int s, int e) -> int {
        int rc;
        hipSetDevice(L.device);
        // slots for this chunk (the lane's previous chunk's copies finish first when it runs dry)
        for (int p = s; p < e; p++) {
            if (L.free_slots.empty() && (rc = complete_pending(L)) != MP2VG_OK) return rc;
            if (L.free_slots.empty()) {
                set_error("frame slot pool exhausted (a picture references a picture outside its chunk window)");
                return MP2VG_E_STATE;
            }
            slot_of[p] = L.free_slots.back();
            L.free_slots.pop_back();
        }
        // chunk records with physical slots; MB and coefficient offsets local to the chunk,
        // gathered straight into pinned memory
        cp.assign(pics + s, pics + e);
        tc = now_ms();
        size_t nc = 0;
        for (int p = s; p < e; p++) {
            if ((rc = parse_session_wait(ps, p)) != MP2VG_OK) return rc;
            ncoef_of[p - s] = parse_session_ncoefs(ps, p);
            nc += ncoef_of[p - s];
        }
        t_wait += now_ms() - tc;
        const size_t nm = (size_t)(e - s) * mbs_per_pic;
        tc = now_ms();
        // this chunk's buffer set fed the lane's upload two chunks back: its copies must have landed
        const int hb = ctx_next_bank(L.ctx);
        if ((rc = ctx_wait_upload(L.ctx, hb)) != MP2VG_OK) return rc;
        if (nc >= (1ull << 32) || !L.mbuf[hb].reserve(nm * sizeof(mp2vg_mb_t)) ||
            !L.cbuf[hb].reserve(std::max<size_t>(nc, 1) * 4))
            return MP2VG_E_NOMEM;
        auto* cm = (mp2vg_mb_t*)L.mbuf[hb].p;
        auto* cc = (uint32_t*)L.cbuf[hb].p;
        for (int i = 0, base = 0; i < e - s; base += (int)ncoef_of[i], i++) base_of[i] = (uint32_t)base;
        parallel_for(e - s, 8, [&](int i) {
            parse_session_append(ps, s + i, cm + (size_t)i * mbs_per_pic, cc + base_of[i], base_of[i]);
        });
        for (int i = 0; i < e - s; i++) {
            mp2vg_picture_t& P = cp[i];
            if (foreign(s + i, P.fwd_slot)) {
                const mp2vg_mb_t* m = cm + (size_t)i * mbs_per_pic;
                for (uint64_t k = 0; k < mbs_per_pic; k++)
                    if (!(m[k].flags & MP2VG_MB_INTRA) && ((m[k].flags & MP2VG_MB_FWD) || !(m[k].flags & MP2VG_MB_BWD))) {
                        set_error("a B picture of a closed GOP predicts forward across GOPs: decode it on one device");
                        return MP2VG_E_UNSUPPORTED;
                    }
                P.fwd_slot = -1;
            }
            P.dst_slot = slot_of[P.dst_slot];
            if (P.fwd_slot >= 0) P.fwd_slot = slot_of[P.fwd_slot];
            if (P.bwd_slot >= 0) P.bwd_slot = slot_of[P.bwd_slot];
            P.mb_first = (uint32_t)((P.mb_first / mbs_per_pic - (uint64_t)s) * mbs_per_pic);
        }
        t_gather += now_ms() - tc;
        tc = now_ms();
        rc = batch_upload_pinned(L.ctx, cp.data(), (int32_t)cp.size(), cm, nm, cc, nc);
        t_up += now_ms() - tc;
        tc = now_ms();
        if (rc == MP2VG_OK) rc = mp2vg_batch_decode(L.ctx);
        if (rc == MP2VG_OK && hipEventRecord(L.decoded, ctx_stream(L.ctx)) != hipSuccess) rc = MP2VG_E_HIP;
        t_dec += now_ms() - tc;
        if (rc != MP2VG_OK) return rc;
        for (int p = s; p < e; p++) queued[p] = 1;
        L.frames += e - s;
        if ((rc = complete_pending(L)) != MP2VG_OK) return rc;
        // copies of this chunk into frame_c-layout frames, one DMA per slot, after its decode
        hipSetDevice(L.device);
        for (int i = 0; i < L.ndl; i++)
            if (hipStreamWaitEvent(L.dl[i], L.decoded, 0) != hipSuccess) return MP2VG_E_HIP;
        FramePool& pool = d->device_frames ? *L.dpool : *d->hpool;
        FrameCopy fc;
        int nfc = 0;
        auto flush_copies = [&]() -> int {
            if (nfc && launch_frame_copy(fc, nfc, d->g.slot_bytes, L.dl[0]) != hipSuccess) {
                set_error("frame copy kernel launch failed");
                return MP2VG_E_HIP;
            }
            nfc = 0;
            return MP2VG_OK;
        };
        for (int p = s; p < e; p++) {
            HostFrame* hf = pool.get(renderer_holds);
            if (!hf) return MP2VG_E_NOMEM;
            for (int i = 0; i < 3; i++) {
                hf->f.planes[i] = hf->data + d->g.plane_off[i];
                hf->f.width[i] = d->g.pw[i];
                hf->f.height[i] = d->g.ph[i];
                hf->f.stride[i] = d->g.stride[i];
            }
            hf->f.picture_coding_type = pics[p].picture_coding_type;
            hf->f.decode_index = p;
            hf->f.device = L.device;
            void* src = nullptr;
            rc = mp2vg_slot_device_ptr(L.ctx, slot_of[p], &src);
            hipSetDevice(L.device);
            // the pinned frame as this device addresses it (a frame the device cannot map goes
            // by DMA)
            // (device frames: the frame itself, in HBM on this lane's device)
            void* hdst = d->device_frames ? (void*)hf->data : nullptr;
            const bool by_kernel = d->kernel_copy &&
                                   (d->device_frames || hipHostGetDevicePointer(&hdst, hf->data, 0) == hipSuccess) &&
                                   !(((uintptr_t)hdst | (uintptr_t)src) & 15);
            if (rc == MP2VG_OK && by_kernel) {
                fc.src[nfc] = (const uint8_t*)src;
                fc.dst[nfc++] = (uint8_t*)hdst;
                L.inflight[p] = hf;
                if (nfc == kFrameCopyMax && (rc = flush_copies()) != MP2VG_OK) return rc;
                continue;
            }
            if (rc == MP2VG_OK && hipMemcpyAsync(hf->data, src, d->g.slot_bytes,
                                                 d->device_frames ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                                                 L.dl[p % L.ndl]) != hipSuccess)
                rc = MP2VG_E_HIP;
            if (rc != MP2VG_OK) {
                hf->owner->put(hf);
                return rc;
            }
            L.inflight[p] = hf;
        }
        if ((rc = flush_copies()) != MP2VG_OK) return rc;
        L.pend.clear();
        for (int p = s; p < e; p++) L.pend.push_back(p);
        return MP2VG_OK;
    };

    // a lane's pending chunk is completed without blocking when its downloads have all landed
    auto try_complete = [&](Lane& X) -> int {
        if (X.pend.empty()) return MP2VG_OK;
        hipSetDevice(X.device);
        for (int i = 0; i < X.ndl; i++) {
            const hipError_t q = hipStreamQuery(X.dl[i]);
            if (q == hipErrorNotReady) return 1;
            if (q != hipSuccess) return MP2VG_E_HIP;
        }
        return complete_pending(X);
    };
    // chunks: up to kChunk consecutive pictures of one lane; with several lanes a chunk also ends
    // where the stream moves to the next shard's lane, so the chunks (and the parse window) still
    // advance in decode order and every lane decodes while the next one is being fed
    Lane* prev = nullptr;
    uint64_t seq = 0;
    d->handoffs_in_flight = d->handoff_blocks = d->handoffs_landed = d->lane_changes = 0;
    for (int s = 0; s < npics;) {
        Lane& L = lane_of(s);
        int e = s + 1;
        while (e < npics && e - s < kChunk && (nl == 1 || &lane_of(e) == &L)) e++;
        // other lanes whose downloads have landed hand their frames on (display order) without a
        // wait; one still downloading keeps its chunk in flight while this lane is fed, so with
        // several lanes every lane's chunk can be in flight at once.  Only when the frame pool
        // could not give this chunk its frames without growing does the host wait, for the
        // oldest pending lane first (its frames come first in display order).
        const bool change = nl > 1 && prev && prev != &L;
        // a lane change is counted once: the lane just left had nothing in flight or its downloads
        // had landed (non-blocking check: `landed`), it is left in flight, or the host waited for it
        bool landed = change && prev->pend.empty();
        if (nl > 1) {
            for (auto& Xp : d->lanes) {
                const bool was = change && Xp.get() == prev && !Xp->pend.empty();
                if (Xp.get() != &L && (rc = try_complete(*Xp)) < 0) return finish(rc);
                if (was && Xp->pend.empty()) landed = true;
            }
            FramePool& pool = d->device_frames ? *L.dpool : *d->hpool;
            for (;;) {
                if (pool.free_count() >= (size_t)(e - s)) break;
                Lane* old = nullptr;
                for (auto& Xp : d->lanes)
                    if (Xp.get() != &L && !Xp->pend.empty() && (!old || Xp->pend_seq < old->pend_seq)) old = Xp.get();
                if (!old) break;
                d->handoff_blocks++;
                if ((rc = complete_pending(*old)) != MP2VG_OK) return finish(rc);
            }
        }
        if ((rc = run_chunk(L, s, e)) != MP2VG_OK) return finish(rc);
        L.pend_seq = seq++;
        if (change) {
            d->lane_changes++;
            if (!prev->pend.empty()) d->handoffs_in_flight++;
            else if (landed) d->handoffs_landed++;
        }
        prev = &L;
        s = e;
    }
    for (auto& Lp : d->lanes)
        if ((rc = complete_pending(*Lp)) != MP2VG_OK) return finish(rc);
    if (next_display != display.size()) set_error("frames left undelivered in display order");
    rc = finish(next_display == display.size() ? MP2VG_OK : MP2VG_E_STATE);
    trace_phase("dropin: parse wait (sum)", now_ms() - t_wait);
    trace_phase("dropin: gather (sum)", now_ms() - t_gather);
    trace_phase("dropin: upload (sum)", now_ms() - t_up);
    trace_phase("dropin: decode issue (sum)", now_ms() - t_dec);
    trace_phase("dropin: download wait (sum)", now_ms() - t_down);
    trace_phase("dropin: after parse", t0);
    return rc;
}
