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
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

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

// Host frames live in pinned memory, in the device slot layout (= the reference frame_c layout),
// so a decoded slot comes back with one contiguous DMA copy (with MP2VG_DECODER_DEVICE_FRAMES
// they are HBM buffers and the copy is device to device, no PCIe).  They are recycled after the render
// callback returns (a frame is valid only during the callback, reference threads.cpp:75-80).
// The pool belongs to the decoder and is filled when it is created, as the reference allocates
// its picture pool up front (decoder.cpp:381-406).
struct HostFrame {
    uint8_t* data = nullptr;
    mp2vg_frame_t f;
};

class FramePool {
  public:
    FramePool(size_t bytes, bool device) : bytes_(bytes), device_(device) {}
    ~FramePool() {
        for (HostFrame* f : all_) {
            if (device_)
                hipFree(f->data);
            else
                hipHostFree(f->data);
            delete f;
        }
    }
    bool reserve(int n) {
        while ((int)all_.size() < n) {
            HostFrame* f = alloc();
            if (!f) return false;
            put(f);
        }
        return true;
    }
    HostFrame* get() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (!free_.empty()) {
                HostFrame* f = free_.back();
                free_.pop_back();
                return f;
            }
        }
        return alloc();
    }
    void put(HostFrame* f) {
        std::lock_guard<std::mutex> lk(mu_);
        free_.push_back(f);
    }

  private:
    HostFrame* alloc() {
        auto* f = new HostFrame();
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
    std::mutex mu_;
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
}  // namespace

struct mp2vg_decoder {
    mp2vg_config_t cfg{};
    mp2vg_render_fn fn = nullptr;
    void* user = nullptr;
    mp2vg_ctx_t* ctx = nullptr;
    Geom g{};
    int nslots = 0;
    std::unique_ptr<FramePool> pool;
    PinnedBuf mbuf[2], cbuf[2];        // chunk MB records / coefficient words, one set per record bank
    // frame downloads, slots dealt round-robin: each stream's copies go to their own DMA engine
    hipStream_t dl[kMaxDl] = {};
    int ndl = 1;
    hipEvent_t decoded = nullptr;      // end of the last chunk's decode (on the context stream)
    bool device_frames = false;        // MP2VG_DECODER_DEVICE_FRAMES: frames handed over in HBM
};

extern "C" int mp2vg_decoder_destroy(mp2vg_decoder_t* d) {
    if (!d) return MP2VG_E_INVALID;
    for (hipStream_t st : d->dl)
        if (st) hipStreamSynchronize(st);
    if (d->ctx) mp2vg_synchronize(d->ctx);
    d->pool.reset();
    if (d->decoded) hipEventDestroy(d->decoded);
    for (hipStream_t st : d->dl)
        if (st) hipStreamDestroy(st);
    if (d->ctx) mp2vg_destroy(d->ctx);
    delete d;
    return MP2VG_OK;
}

extern "C" int mp2vg_decoder_create(const mp2vg_config_t* cfg, mp2vg_render_fn fn, void* user,
                                    mp2vg_decoder_t** out) {
    if (!cfg || !fn || !out) return MP2VG_E_INVALID;
    *out = nullptr;
    if (cfg->reserved & ~MP2VG_DECODER_DEVICE_FRAMES) {
        set_error("unknown decoder flags in mp2vg_config_t.reserved");
        return MP2VG_E_INVALID;
    }
    mp2vg_config_t c = *cfg;
    // chunk k decodes into its own slots while chunk k-1 is still being downloaded
    c.pictures_pool_size = std::max(cfg->pictures_pool_size, 2 * kChunk + 4);
    mp2vg_ctx_t* ctx = nullptr;
    int rc = mp2vg_create(&c, &ctx);
    if (rc != MP2VG_OK) return rc;
    auto* d = new mp2vg_decoder();
    d->cfg = c;
    d->fn = fn;
    d->user = user;
    d->ctx = ctx;
    d->g.init(c.width, c.height, c.chroma_format);
    d->nslots = c.pictures_pool_size;
    d->device_frames = c.reserved & MP2VG_DECODER_DEVICE_FRAMES;
    d->pool.reset(new FramePool(d->g.slot_bytes, d->device_frames));
    ctx_set_launch_timing(ctx, false);  // no per-launch events on the drop-in's chunk path
    d->ndl = kDlStreams;
    bool sok = true;
    for (int i = 0; i < d->ndl; i++) sok = sok && hipStreamCreateWithFlags(&d->dl[i], hipStreamNonBlocking) == hipSuccess;
    if (!sok ||
        hipEventCreateWithFlags(&d->decoded, hipEventDisableTiming) != hipSuccess) {
        set_error("download stream / event creation failed");
        mp2vg_decoder_destroy(d);
        return MP2VG_E_HIP;
    }
    // chunk record buffers sized up front: every MB record of a chunk, and 32 coefficient words
    // per MB (the bench stream needs 12.5; a chunk that needs more grows its set once)
    const size_t chunk_mbs = (size_t)kChunk * (c.width / 16) * (c.height / 16);
    bool ok = true;
    for (int i = 0; i < 2; i++)
        ok = ok && d->mbuf[i].reserve(chunk_mbs * sizeof(mp2vg_mb_t)) && d->cbuf[i].reserve(chunk_mbs * 32 * 4);
    // frames in flight: one chunk being copied, one being rendered, anchors held for display
    if (!ok || !d->pool->reserve(2 * kChunk + 4)) {
        set_error("pinned host frame allocation failed");
        mp2vg_decoder_destroy(d);
        return MP2VG_E_NOMEM;
    }
    *out = d;
    return MP2VG_OK;
}

extern "C" int mp2vg_decoder_decode(mp2vg_decoder_t* d, const uint8_t* buf, uint64_t len) {
    if (!d || !buf) return MP2VG_E_INVALID;
    // the parse runs on worker threads while the chunks below go through the device: a chunk
    // waits only for its own pictures (two threads are left for this loop and the renderer)
    double t0 = now_ms(), tc;
    double t_up = 0, t_dec = 0, t_down = 0, t_wait = 0, t_gather = 0;
    ParseSession* ps = nullptr;
    const int threads = d->cfg.num_threads > 0 ? d->cfg.num_threads : (int)std::thread::hardware_concurrency();
    // (16-thread box: 2 or 4 threads kept back 1,975 frames/s, 1 -> 1,864, 6 -> 1,661)
    int rc = parse_session_start(buf, len, &d->cfg, std::max(1, threads - 2), 4 * kChunk, &ps);
    t0 = trace_phase("dropin: headers", t0);
    if (rc != MP2VG_OK) return rc;
    std::unique_ptr<ParseSession, void (*)(ParseSession*)> guard(ps, parse_session_free);
    const int32_t npics = parse_session_npics(ps);
    const mp2vg_picture_t* pics = parse_session_pictures(ps);
    std::vector<int32_t> display(parse_session_display(ps), parse_session_display(ps) + npics);

    // last decode index that predicts from each picture
    std::vector<int> last_use(npics, -1);
    for (int q = 0; q < npics; q++) {
        if (pics[q].fwd_slot >= 0) last_use[pics[q].fwd_slot] = q;
        if (pics[q].bwd_slot >= 0) last_use[pics[q].bwd_slot] = q;
    }

    // render thread (decoder.cpp:403, :346-379)
    std::mutex mu;
    std::condition_variable cv;
    std::deque<HostFrame*> q;
    bool done = false;
    FramePool& pool = *d->pool;
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
            pool.put(f);
        }
    });

    std::vector<int> slot_of(npics, -1);
    std::vector<int> free_slots;
    for (int s = d->nslots - 1; s >= 0; s--) free_slots.push_back(s);
    std::map<int, HostFrame*> ready;  // decode index -> downloaded frame
    size_t next_display = 0;
    std::vector<mp2vg_picture_t> cp;
    std::vector<size_t> ncoef_of(kChunk);
    std::vector<uint32_t> base_of(kChunk);
    const uint64_t mbs_per_pic = (uint64_t)(d->cfg.width / 16) * (d->cfg.height / 16);

    auto finish = [&](int status) {
        for (int i = 0; i < d->ndl; i++) hipStreamSynchronize(d->dl[i]);  // no copy may still target a pool frame
        mp2vg_synchronize(d->ctx);
        {
            std::lock_guard<std::mutex> lk(mu);
            done = true;
        }
        cv.notify_all();
        render.join();
        return status;
    };

    // Chunk pipeline, nothing waits for the device except through an event:
    //   host:   gather chunk k's records (pinned) | upload (copy stream; waits only for the decode
    //           of chunk k-2, which read the same record bank) | queue decode k | complete k-1
    //   device: decode k-1 ... decode k (context stream) while the D2H copies of k-1 run (dl)
    // A chunk's frames reach the renderer, and its slots return to the free list, only after its
    // copies have completed; a released slot is rewritten only by a later chunk, whose decode is
    // ordered after every earlier decode on the context stream.
    std::map<int, HostFrame*> inflight;  // decode index -> frame whose copy is in flight
    int pend_e = -1;                     // end of the chunk whose copies are in flight
    int decoded_e = 0;                   // the decodes of pictures [0, decoded_e) are queued
    auto complete_pending = [&]() -> int {
        if (pend_e < 0) return MP2VG_OK;
        tc = now_ms();
        for (int i = 0; i < d->ndl; i++)
            if (hipStreamSynchronize(d->dl[i]) != hipSuccess) return MP2VG_E_HIP;
        t_down += now_ms() - tc;
        for (auto& kv : inflight) ready[kv.first] = kv.second;
        inflight.clear();
        // release slots no later picture predicts from
        for (int p = 0; p < pend_e; p++)
            if (slot_of[p] >= 0 && last_use[p] < decoded_e) {
                free_slots.push_back(slot_of[p]);
                slot_of[p] = -1;
            }
        pend_e = -1;
        // hand frames to the render thread in display order
        while (next_display < display.size() && ready.count(display[next_display])) {
            auto it = ready.find(display[next_display]);
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

    for (int s = 0; s < npics; s += kChunk) {
        int e = std::min(npics, s + kChunk);
        // slots for this chunk (the previous chunk's copies finish first when the pool runs dry)
        for (int p = s; p < e; p++) {
            if (free_slots.empty() && (rc = complete_pending()) != MP2VG_OK) return finish(rc);
            if (free_slots.empty()) return finish(MP2VG_E_STATE);
            slot_of[p] = free_slots.back();
            free_slots.pop_back();
        }
        // chunk records with physical slots; MB and coefficient offsets local to the chunk,
        // gathered straight into pinned memory
        cp.assign(pics + s, pics + e);
        tc = now_ms();
        size_t nc = 0;
        for (int p = s; p < e; p++) {
            if ((rc = parse_session_wait(ps, p)) != MP2VG_OK) return finish(rc);
            ncoef_of[p - s] = parse_session_ncoefs(ps, p);
            nc += ncoef_of[p - s];
        }
        t_wait += now_ms() - tc;
        const size_t nm = (size_t)(e - s) * mbs_per_pic;
        tc = now_ms();
        // this chunk's buffer set fed the upload two chunks back: its copies must have landed
        const int hb = ctx_next_bank(d->ctx);
        if ((rc = ctx_wait_upload(d->ctx, hb)) != MP2VG_OK) return finish(rc);
        if (nc >= (1ull << 32) || !d->mbuf[hb].reserve(nm * sizeof(mp2vg_mb_t)) ||
            !d->cbuf[hb].reserve(std::max<size_t>(nc, 1) * 4))
            return finish(MP2VG_E_NOMEM);
        auto* cm = (mp2vg_mb_t*)d->mbuf[hb].p;
        auto* cc = (uint32_t*)d->cbuf[hb].p;
        for (int i = 0, base = 0; i < e - s; base += (int)ncoef_of[i], i++) base_of[i] = (uint32_t)base;
        parallel_for(e - s, 8, [&](int i) {
            parse_session_append(ps, s + i, cm + (size_t)i * mbs_per_pic, cc + base_of[i], base_of[i]);
        });
        for (auto& P : cp) {
            P.dst_slot = slot_of[P.dst_slot];
            if (P.fwd_slot >= 0) P.fwd_slot = slot_of[P.fwd_slot];
            if (P.bwd_slot >= 0) P.bwd_slot = slot_of[P.bwd_slot];
            P.mb_first = (uint32_t)((P.mb_first / mbs_per_pic - (uint64_t)s) * mbs_per_pic);
        }
        t_gather += now_ms() - tc;
        tc = now_ms();
        rc = batch_upload_pinned(d->ctx, cp.data(), (int32_t)cp.size(), cm, nm, cc, nc);
        t_up += now_ms() - tc;
        tc = now_ms();
        if (rc == MP2VG_OK) rc = mp2vg_batch_decode(d->ctx);
        if (rc == MP2VG_OK && hipEventRecord(d->decoded, ctx_stream(d->ctx)) != hipSuccess) rc = MP2VG_E_HIP;
        t_dec += now_ms() - tc;
        if (rc != MP2VG_OK) return finish(rc);
        decoded_e = e;
        if ((rc = complete_pending()) != MP2VG_OK) return finish(rc);
        // copies of this chunk into frame_c-layout host frames, one DMA per slot, after its decode
        for (int i = 0; i < d->ndl; i++)
            if (hipStreamWaitEvent(d->dl[i], d->decoded, 0) != hipSuccess) return finish(MP2VG_E_HIP);
        for (int p = s; p < e; p++) {
            HostFrame* hf = pool.get();
            if (!hf) return finish(MP2VG_E_NOMEM);
            for (int i = 0; i < 3; i++) {
                hf->f.planes[i] = hf->data + d->g.plane_off[i];
                hf->f.width[i] = d->g.pw[i];
                hf->f.height[i] = d->g.ph[i];
                hf->f.stride[i] = d->g.stride[i];
            }
            hf->f.picture_coding_type = pics[p].picture_coding_type;
            hf->f.decode_index = p;
            void* src = nullptr;
            rc = mp2vg_slot_device_ptr(d->ctx, slot_of[p], &src);
            if (rc == MP2VG_OK && hipMemcpyAsync(hf->data, src, d->g.slot_bytes,
                                                 d->device_frames ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                                                 d->dl[p % d->ndl]) != hipSuccess)
                rc = MP2VG_E_HIP;
            if (rc != MP2VG_OK) {
                pool.put(hf);
                return finish(rc);
            }
            inflight[p] = hf;
        }
        pend_e = e;
    }
    if ((rc = complete_pending()) != MP2VG_OK) return finish(rc);
    rc = finish(next_display == display.size() ? MP2VG_OK : MP2VG_E_STATE);
    trace_phase("dropin: parse wait (sum)", now_ms() - t_wait);
    trace_phase("dropin: gather (sum)", now_ms() - t_gather);
    trace_phase("dropin: upload (sum)", now_ms() - t_up);
    trace_phase("dropin: decode issue (sum)", now_ms() - t_dec);
    trace_phase("dropin: download wait (sum)", now_ms() - t_down);
    trace_phase("dropin: after parse", t0);
    return rc;
}
