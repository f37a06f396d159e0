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

namespace {
constexpr int kChunk = 16;  // pictures per device batch

// Host frames live in pinned memory, in the device slot layout (= the reference frame_c layout),
// so a decoded slot comes back with one contiguous DMA copy.  They are recycled after the render
// callback returns (a frame is valid only during the callback, reference threads.cpp:75-80).
struct HostFrame {
    uint8_t* data = nullptr;
    mp2vg_frame_t f;
};

class FramePool {
  public:
    explicit FramePool(size_t bytes) : bytes_(bytes) {}
    ~FramePool() {
        for (HostFrame* f : all_) {
            hipHostFree(f->data);
            delete f;
        }
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
        auto* f = new HostFrame();
        if (hipHostMalloc((void**)&f->data, bytes_, hipHostMallocDefault) != hipSuccess) {
            delete f;
            return nullptr;
        }
        std::lock_guard<std::mutex> lk(mu_);
        all_.push_back(f);
        return f;
    }
    void put(HostFrame* f) {
        std::lock_guard<std::mutex> lk(mu_);
        free_.push_back(f);
    }

  private:
    size_t bytes_;
    std::mutex mu_;
    std::vector<HostFrame*> all_, free_;
};
}  // namespace

struct mp2vg_decoder {
    mp2vg_config_t cfg{};
    mp2vg_render_fn fn = nullptr;
    void* user = nullptr;
    mp2vg_ctx_t* ctx = nullptr;
    Geom g{};
    int nslots = 0;
};

extern "C" int mp2vg_decoder_create(const mp2vg_config_t* cfg, mp2vg_render_fn fn, void* user,
                                    mp2vg_decoder_t** out) {
    if (!cfg || !fn || !out) return MP2VG_E_INVALID;
    *out = nullptr;
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
    *out = d;
    return MP2VG_OK;
}

extern "C" int mp2vg_decoder_destroy(mp2vg_decoder_t* d) {
    if (!d) return MP2VG_E_INVALID;
    mp2vg_destroy(d->ctx);
    delete d;
    return MP2VG_OK;
}

extern "C" int mp2vg_decoder_decode(mp2vg_decoder_t* d, const uint8_t* buf, uint64_t len) {
    if (!d || !buf) return MP2VG_E_INVALID;
    // the parse runs on worker threads while the chunks below go through the device: a chunk
    // waits only for its own pictures (two threads are left for this loop and the renderer)
    double t0 = now_ms(), tc;
    double t_up = 0, t_dec = 0, t_down = 0, t_wait = 0;
    ParseSession* ps = nullptr;
    const int threads = d->cfg.num_threads > 0 ? d->cfg.num_threads : (int)std::thread::hardware_concurrency();
    // (16-thread box: 2 or 4 threads kept back 1,975 frames/s, 1 -> 1,864, 6 -> 1,661)
    int rc = parse_session_start(buf, len, &d->cfg, std::max(1, threads - 2), &ps);
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
    FramePool pool(d->g.slot_bytes);
    hipStream_t dl = nullptr;
    if (hipStreamCreateWithFlags(&dl, hipStreamNonBlocking) != hipSuccess) return MP2VG_E_HIP;
    std::unique_ptr<void, void (*)(void*)> dl_guard(dl, [](void* s) { hipStreamDestroy((hipStream_t)s); });
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
    std::vector<mp2vg_mb_t> cm;
    std::vector<uint32_t> cc;
    const uint64_t mbs_per_pic = (uint64_t)(d->cfg.width / 16) * (d->cfg.height / 16);

    auto finish = [&](int status) {
        hipStreamSynchronize(dl);  // no copy may still target a pool frame
        {
            std::lock_guard<std::mutex> lk(mu);
            done = true;
        }
        cv.notify_all();
        render.join();
        return status;
    };

    // Chunk pipeline: the D2H copies of chunk k-1 (stream dl) run while chunk k is uploaded and
    // decoded.  A chunk's frames reach the renderer, and its slots return to the free list, only
    // after its copies have completed.
    std::map<int, HostFrame*> inflight;  // decode index -> frame whose copy is in flight
    int pend_e = -1;                     // end of the chunk whose copies are in flight
    int decoded_e = 0;                   // pictures [0, decoded_e) are decoded
    auto complete_pending = [&]() -> int {
        if (pend_e < 0) return MP2VG_OK;
        tc = now_ms();
        if (hipStreamSynchronize(dl) != hipSuccess) return MP2VG_E_HIP;
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
        // chunk records with physical slots; MB and coefficient offsets local to the chunk
        cp.assign(pics + s, pics + e);
        cm.resize((size_t)(e - s) * mbs_per_pic);
        cc.clear();
        tc = now_ms();
        for (int p = s; p < e; p++) {
            if ((rc = parse_session_wait(ps, p)) != MP2VG_OK) return finish(rc);
            parse_session_append(ps, p, cm.data() + (size_t)(p - s) * mbs_per_pic, cc);
        }
        t_wait += now_ms() - tc;
        for (auto& P : cp) {
            P.dst_slot = slot_of[P.dst_slot];
            if (P.fwd_slot >= 0) P.fwd_slot = slot_of[P.fwd_slot];
            if (P.bwd_slot >= 0) P.bwd_slot = slot_of[P.bwd_slot];
            P.mb_first = (uint32_t)((P.mb_first / mbs_per_pic - (uint64_t)s) * mbs_per_pic);
        }
        tc = now_ms();
        rc = mp2vg_batch_upload(d->ctx, cp.data(), (int32_t)cp.size(), cm.data(), cm.size(), cc.data(), cc.size());
        t_up += now_ms() - tc;
        tc = now_ms();
        if (rc == MP2VG_OK) rc = mp2vg_batch_decode(d->ctx);
        if (rc == MP2VG_OK) rc = mp2vg_synchronize(d->ctx);
        t_dec += now_ms() - tc;
        if (rc != MP2VG_OK) return finish(rc);
        decoded_e = e;
        if ((rc = complete_pending()) != MP2VG_OK) return finish(rc);
        // copies of this chunk into frame_c-layout host frames: one DMA per slot
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
            if (rc == MP2VG_OK && hipMemcpyAsync(hf->data, src, d->g.slot_bytes, hipMemcpyDeviceToHost, dl) != hipSuccess)
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
    trace_phase("dropin: upload (sum)", now_ms() - t_up);
    trace_phase("dropin: decode (sum)", now_ms() - t_dec);
    trace_phase("dropin: download (sum)", now_ms() - t_down);
    trace_phase("dropin: after parse", t0);
    return rc;
}
