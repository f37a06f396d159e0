// runtime.cpp — device context of the C ABI: frame pool in HBM, resident record batch, the
// dependency-level scheduler (one kernel launch per level), timing, downloads and digests.
//
// Replaces the reference's frame pool + task DAG (decoder.cpp:381-406, threads.cpp:22-211): a
// picture's slices become workgroups; pictures whose references are complete run together in
// one launch, so a batch of closed GOPs needs only as many launches as its longest
// I->P->...->B chain.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include <atomic>
#include <thread>

#include "recon_kernel.h"
#include "syntax.h"

namespace mp2vg {
hipError_t launch_recon(int cf, int mcm, const KArgs& a, hipStream_t stream);
hipError_t launch_tile_convert(const KArgs& a, int cf, const int32_t* d_list, int n, int32_t slot0, hipStream_t stream);
hipError_t launch_clock_probe(unsigned long long* d_out, int iters, int blocks, hipStream_t stream);
hipError_t launch_block_probe(void* p, size_t bytes, int rw, int reps, void* sink, hipStream_t stream);
hipError_t launch_block_random(const void* base, size_t bytes, int waves, int iters, void* sink, hipStream_t stream);
hipError_t launch_pool_scatter(const uint64_t* tab, int nslots, uint32_t fkb, uint32_t tkb, int lock, int waves,
                               int iters, void* sink, hipStream_t stream);
hipError_t launch_digest(const uint64_t* ftab, const int32_t* d_slots, int n,
                         const uint64_t off[3], const int32_t stride[3], const int32_t w[3],
                         const int32_t h[3], unsigned long long* d_out, hipStream_t stream);
}  // namespace mp2vg

using namespace mp2vg;

#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                  \
            return MP2VG_E_HIP;                                                            \
        }                                                                                  \
    } while (0)

static constexpr size_t kPoolPad = 4096 + 65536;  // slack after the last slot: clamped row over-reads, the
                                                  // kernel's dummy load / store sink at +2048 (kSinkOff) and,
                                                  // from +4096, one 64-B sink line per wave (1024 lines)
static constexpr size_t kSinkOff = 2048;
static constexpr size_t kCoefPad = 256;        // the kernel prefetches up to 256 coefficient words per MB group
static constexpr size_t kStageBytes = 32u << 20;
static constexpr size_t kMbPad = 16;  // >= the kernel's MB group size
// independent picture sets per batch, one stream each (c2: 1 set 2.575 ms, 2 sets 2.502-2.535 ms,
// 3 sets 2.566, 4 sets 2.590; MP2VG_STREAMS overrides for measurements)
static int default_streams(const mp2vg_config_t* cfg) {
    if (cfg->reserved & MP2VG_CTX_ONE_STREAM) return 1;
    const char* e = getenv("MP2VG_STREAMS");
    return e ? std::max(1, atoi(e)) : 2;
}
// how the picture sets' launch chains are coupled inside a batch (MP2VG_SET_COUPLE overrides for
// measurements): 0 free-running streams; 1 lockstep (launch k of a set waits for launch k-1 of
// every other set); 2 staggered (set s > 0 runs launch k after set s-1's launch k, and set s-1's
// launch k+1 waits for set s's launch k-1: set s trails by one to two launches)
// Bytes between consecutive frame slots beyond the slot itself (MP2VG_SLOT_PAD overrides for the
// pool-placement measurements, profiles/r4/README.md): slot offsets decide which HBM channels the
// same pixel rows of different pictures land on.
// (Dev builds only, -DMP2VG_DEV_ABLATIONS: a product library ignores these variables.)
static const char* dev_env(const char* name) {
#ifdef MP2VG_DEV_ABLATIONS
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}
static void pool_block_free(uint8_t* p, size_t bytes, uint64_t vmm);
static void free_held_pools(mp2vg_ctx_t* c);
static size_t slot_pad() {
    const char* e = dev_env("MP2VG_SLOT_PAD");
    return e ? (size_t)std::max(0, atoi(e)) & ~(size_t)255 : 0;
}
static size_t tile_pad() {  // the same for the anchor-tile slots (MP2VG_TILE_PAD)
    const char* e = dev_env("MP2VG_TILE_PAD");
    return e ? (size_t)std::max(0, atoi(e)) & ~(size_t)255 : 0;
}
static int set_coupling() {
    const char* e = dev_env("MP2VG_SET_COUPLE");
    return e ? atoi(e) : 0;
}

// Which pictures of a batch write anchor tiles (recon.hip tile_off: the taps read references from
// them), decided per batch by plan_batch: a picture does when a later picture of the batch reads
// its slot, or when it is one of the batch's last two I/P pictures (the next batch's first
// pictures may predict from those: references are the two latest anchors, decoder.cpp:299-304).
// A reference slot that the batch reads before writing it must hold tiles from an earlier batch;
// when its tiles are stale (its writer did not store them) mp2vg_batch_decode rebuilds them from
// the frame (tile_convert) on the reading set's stream first.  The I and P loops store their
// tiles themselves (building every I picture's tiles by conversion after its launch measured c2
// -2.3 %), except in I-only launches where few pictures store tiles (mode 4, plan_batch); B
// pictures that a later picture reads (never in an MPEG-2 stream) and those I pictures get theirs
// from tile_convert right after their launch, one launch over its pictures.
struct TilePlan {
    std::vector<std::pair<int32_t, int32_t>> ext_reads;  // (slot, set) read before written
    std::vector<std::pair<int32_t, uint8_t>> writes;     // (slot, tiles written) in decode order
    std::vector<std::pair<int32_t, int32_t>> post;       // (launch, slot): B pictures read later
};

// One resident record batch.  The context keeps two, so the upload of batch k+1 (on the copy
// stream) overlaps the decode of batch k; an upload waits only for the decode that last read
// the bank it overwrites (batch k-1).
struct Bank {
    mp2vg_picture_t* d_pics = nullptr;
    size_t cap_pics = 0;
    mp2vg_mb_t* d_mbs = nullptr;
    size_t cap_mbs = 0;
    uint32_t* d_coefs = nullptr;
    size_t cap_coefs = 0;
    SliceDesc* d_slices = nullptr;
    size_t cap_slices = 0;
    int32_t* d_post = nullptr;  // TilePlan.post slots, in launch order (post_of[i]: launch i's range)
    size_t cap_post = 0;
    // pinned staging of the bank's small arrays (pictures, slices, post lists) for the
    // asynchronous uploads of the drop-in decoder: copied without a host wait
    uint8_t* h_small = nullptr;
    size_t cap_small = 0;
    std::vector<std::pair<int32_t, int32_t>> post_of;
    std::vector<Launch> launches;  // slice ranges per (dependency level, picture type)
    std::vector<std::vector<int32_t>> foot;  // per picture set: the slots it writes or reads
    TilePlan tiles;
    int32_t npics = 0;
    hipEvent_t uploaded = nullptr;  // on ustream, after the bank's copies
    hipEvent_t consumed = nullptr;  // on stream, after the last decode that read the bank
    bool decoded = false;           // `consumed` has been recorded
};

struct PoolSet;
struct mp2vg_ctx {
    mp2vg_config_t cfg{};
    Geom g{};
    hipStream_t stream = nullptr;  // joins every set of each batch; every API call synchronises on it
    hipStream_t ustream = nullptr;  // record uploads
    std::vector<hipStream_t> sstreams;  // one per picture set (created on first use)
    std::vector<hipEvent_t> sev;        // end of each set's launches in the last batch
    std::vector<hipEvent_t> lev;        // end of each launch of the current batch (set coupling)
    std::vector<std::vector<uint8_t>> last_foot;  // slots each set of the last batch touched
    uint8_t* d_pool = nullptr;   // the frame slots in one block (null with MP2VG_POOL_CHUNK)
    int32_t nslots = 0;
    size_t slot_stride = 0;  // bytes from one slot to the next: the slot size plus slot_pad()
    uint8_t* d_tiles = nullptr;  // anchor tiles of each slot (recon.hip tile_off): the taps' source
    // per-slot device addresses of the frame and of its tiles (host copies, and the table the
    // kernels index: [frames | tiles]); chunked pools (MP2VG_POOL_CHUNK slots per block) add blocks
    std::vector<uint64_t> fptr, tptr;
    std::vector<uint8_t*> chunks;
    std::vector<size_t> chunk_bytes;  // allocation size of each block in `chunks`
    std::vector<uint64_t> chunk_vmm;  // per block: its physical handle when mapped by pool_block_alloc (else 0)
    uint64_t* d_tab = nullptr;
    uint8_t* d_sink = nullptr;   // dummy loads / stores of the kernels (kPoolPad bytes)
    std::vector<uint8_t> tiles_ok;  // per slot: its tiles match its frame (after the batches enqueued)
    size_t tile_stride = 0;      // 2 x slot bytes, 256-B aligned
    int nstreams = 2;  // independent picture sets per batch (default_streams)
    int ncu = 0;       // the device's CUs (0 in a host-only planning shell: 256 assumed)

    Bank bank[2];
    int cur = -1;  // bank of the last upload
    bool batch_ready = false;

    // timing events of the last kHist batches (ring, slot = batch sequence number % kHist), so a
    // caller can decode back to back and read every batch's times afterwards
    struct BatchEv {
        hipEvent_t b[2] = {nullptr, nullptr};  // b[1]: end of the whole batch (main stream)
        std::vector<hipEvent_t> s;             // start of each picture set (on its stream; the
                                               // batch starts at the earliest of them)
        int ns = 0;                            // sets of this batch
        std::vector<hipEvent_t> l;             // 2 per launch (start, end; on the launch's stream)
        int nl = 0;                            // launches timed (0 with launch timing off)
    };
    static constexpr int kHist = 64;
    BatchEv hist[kHist];
    uint64_t seq = 0;  // batches decoded
    hipEvent_t up_ev[2] = {nullptr, nullptr};  // staging halves of upload()
    bool launch_timing = true;  // per-launch events (mp2vg_last_launch_times)
    bool placed = false;        // the pool's placement was calibrated (calibrate_placement)
    std::vector<float> place_ms;  // its batch times: round 0 of every candidate, then round 1
    int place_kept = -1;          // the candidate kept (0 = the pool as first allocated)
    std::vector<PoolSet*> place_held;  // the calibration's candidates not kept, held until destroy

    void* h_stage = nullptr;
    int32_t* d_dslots = nullptr;
    unsigned long long* d_digest = nullptr;
    size_t cap_digest = 0;
};

template <class T>
static int grow(T*& p, size_t& cap, size_t n) {
    if (n <= cap) return MP2VG_OK;
    if (p) HIPCHK(hipFree(p));
    p = nullptr;
    size_t c = std::max(n, cap * 3 / 2);
    HIPCHK(hipMalloc((void**)&p, c * sizeof(T)));
    cap = c;
    return MP2VG_OK;
}

// Host -> device copy on the copy stream.  Pageable sources go through the pinned staging
// buffer, double-buffered (the memcpy of the next half overlaps the DMA of the previous one);
// pinned sources (the drop-in decoder's chunk buffers) are copied directly.  The caller
// synchronises the copy stream before its host buffers may change.
static int upload(mp2vg_ctx_t* ctx, void* dst, const void* src, size_t bytes, bool pinned) {
    if (pinned) {
        if (bytes) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->ustream));
        return MP2VG_OK;
    }
    const uint8_t* s = (const uint8_t*)src;
    uint8_t* d = (uint8_t*)dst;
    const size_t half = kStageBytes / 2;
    for (int i = 0; bytes; i++) {
        const size_t n = std::min(bytes, half);
        uint8_t* st = (uint8_t*)ctx->h_stage + (i & 1) * half;
        if (i >= 2) HIPCHK(hipEventSynchronize(ctx->up_ev[i & 1]));
        memcpy(st, s, n);
        HIPCHK(hipMemcpyAsync(d, st, n, hipMemcpyHostToDevice, ctx->ustream));
        HIPCHK(hipEventRecord(ctx->up_ev[i & 1], ctx->ustream));
        s += n;
        d += n;
        bytes -= n;
    }
    HIPCHK(hipStreamSynchronize(ctx->ustream));
    return MP2VG_OK;
}

extern "C" int mp2vg_create(const mp2vg_config_t* cfg, mp2vg_ctx_t** out) {
    if (!cfg || !out) return MP2VG_E_INVALID;
    *out = nullptr;
    if (mp2vg_frame_geometry(cfg, nullptr, nullptr, nullptr, nullptr) != MP2VG_OK) return MP2VG_E_INVALID;
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (cfg->device < 0 || cfg->device >= ndev) {
        set_error("no such HIP device");
        return MP2VG_E_HIP;
    }
    HIPCHK(hipSetDevice(cfg->device));
    // dev knob (placement study, profiles/r6/README.md): before the process's first context, N
    // helper streams each submit one memset and are kept, so they take the first hardware queues
    if (const char* qw = dev_env("MP2VG_QUEUE_WARM")) {
        static bool warmed = false;
        if (!warmed) {
            warmed = true;
            void* buf = nullptr;
            if (hipMalloc(&buf, 4096) == hipSuccess)
                for (int i = 0; i < atoi(qw); i++) {
                    hipStream_t st;
                    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess)
                        (void)hipMemsetAsync(buf, 0, 4096, st);
                }
            (void)hipDeviceSynchronize();
        }
    }
    mp2vg_ctx_t* c = new mp2vg_ctx_t();
    c->cfg = *cfg;
    c->g.init(cfg->width, cfg->height, cfg->chroma_format);
    c->slot_stride = c->g.slot_bytes + slot_pad();
    c->tile_stride = ((2 * c->g.slot_bytes + 255) & ~(size_t)255) + tile_pad();
    c->nstreams = default_streams(cfg);
    if (hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, cfg->device) != hipSuccess) c->ncu = 0;
    bool ok = true;
    for (Bank& b : c->bank)
        ok = ok && hipEventCreateWithFlags(&b.uploaded, hipEventDisableTiming | hipEventBlockingSync) == hipSuccess &&
             hipEventCreateWithFlags(&b.consumed, hipEventDisableTiming) == hipSuccess;
    if (!ok || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->ustream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->up_ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->up_ev[1], hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc(&c->h_stage, kStageBytes, hipHostMallocDefault) != hipSuccess) {
        set_error("stream / pinned staging allocation failed");
        mp2vg_destroy(c);
        return MP2VG_E_HIP;
    }
    int rc = mp2vg_reserve_slots(c, std::max(1, cfg->pictures_pool_size));
    if (rc != MP2VG_OK) {
        mp2vg_destroy(c);
        return rc;
    }
    *out = c;
    return MP2VG_OK;
}

extern "C" int mp2vg_destroy(mp2vg_ctx_t* c) {
    if (!c) return MP2VG_E_INVALID;
    hipSetDevice(c->cfg.device);
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->ustream) hipStreamSynchronize(c->ustream);
    for (auto& h : c->hist) {
        for (auto e : h.l) hipEventDestroy(e);
        for (auto e : h.s)
            if (e) hipEventDestroy(e);
        for (auto e : h.b)
            if (e) hipEventDestroy(e);
    }
    for (auto e : c->up_ev)
        if (e) hipEventDestroy(e);

    hipFree(c->d_pool);
    hipFree(c->d_tiles);
    for (size_t i = 0; i < c->chunks.size(); i++) pool_block_free(c->chunks[i], c->chunk_bytes[i], c->chunk_vmm[i]);
    free_held_pools(c);
    hipFree(c->d_tab);
    hipFree(c->d_sink);
    for (Bank& b : c->bank) {
        hipFree(b.d_pics);
        hipFree(b.d_mbs);
        hipFree(b.d_coefs);
        hipFree(b.d_slices);
        hipFree(b.d_post);
        if (b.h_small) hipHostFree(b.h_small);
        if (b.uploaded) hipEventDestroy(b.uploaded);
        if (b.consumed) hipEventDestroy(b.consumed);
    }
    hipFree(c->d_dslots);
    hipFree(c->d_digest);
    if (c->h_stage) hipHostFree(c->h_stage);
    for (auto st : c->sstreams) hipStreamSynchronize(st);
    for (auto e : c->sev) hipEventDestroy(e);
    for (auto e : c->lev) hipEventDestroy(e);
    for (auto st : c->sstreams) hipStreamDestroy(st);
    if (c->ustream) hipStreamDestroy(c->ustream);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return MP2VG_OK;
}

// the slot table the kernels index ([frame addresses | tile addresses]) and the slot state
static int finish_reserve(mp2vg_ctx_t* c, int32_t nslots) {
    hipFree(c->d_tab);
    c->d_tab = nullptr;
    HIPCHK(hipMalloc((void**)&c->d_tab, sizeof(uint64_t) * 2 * nslots));
    HIPCHK(hipMemcpyAsync(c->d_tab, c->fptr.data(), sizeof(uint64_t) * nslots, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_tab + nslots, c->tptr.data(), sizeof(uint64_t) * nslots, hipMemcpyHostToDevice,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->tiles_ok.resize(nslots, 1);  // new slots: zero frame, zero tiles
    c->nslots = nslots;
    c->last_foot.clear();  // every set of every batch is done (c->stream joined them)
    return MP2VG_OK;
}

// One pool block.  Default: hipMalloc.  Dev knobs for the placement study (profiles/r6/README.md):
// MP2VG_POOL_POW2=1 rounds the block up to a power of two; MP2VG_POOL_VMM=<MB> maps it with the
// virtual memory API at a VA aligned to that many MB (0 = the block's own power-of-two size).
static hipError_t pool_block_alloc(int device, size_t bytes, uint8_t** p, size_t* got, uint64_t* vmm) {
    *vmm = 0;
    size_t sz = bytes;
    const char* pw = dev_env("MP2VG_POOL_POW2");
    const char* vm = dev_env("MP2VG_POOL_VMM");
    if ((pw && atoi(pw)) || vm) {
        sz = 1;
        while (sz < bytes) sz <<= 1;
    }
    *got = sz;
    if (!vm) return hipMalloc((void**)p, sz);
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    size_t gran = 0;
    hipError_t e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended);
    if (e != hipSuccess) return e;
    sz = (sz + gran - 1) / gran * gran;
    *got = sz;
    const size_t align = atoi(vm) > 0 ? (size_t)atoi(vm) << 20 : sz;
    hipMemGenericAllocationHandle_t h;
    if ((e = hipMemCreate(&h, sz, &prop, 0)) != hipSuccess) return e;
    void* va = nullptr;
    if ((e = hipMemAddressReserve(&va, sz, align, nullptr, 0)) != hipSuccess) {
        hipMemRelease(h);
        return e;
    }
    if ((e = hipMemMap(va, sz, 0, h, 0)) != hipSuccess) {
        hipMemAddressFree(va, sz);
        hipMemRelease(h);
        return e;
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    if ((e = hipMemSetAccess(va, sz, &acc, 1)) != hipSuccess) {
        hipMemUnmap(va, sz);
        hipMemAddressFree(va, sz);
        hipMemRelease(h);
        return e;
    }
    *p = (uint8_t*)va;
    *vmm = (uint64_t)(uintptr_t)h;
    return hipSuccess;
}

static void pool_block_free(uint8_t* p, size_t bytes, uint64_t vmm) {
    if (!vmm) {
        hipFree(p);
        return;
    }
    hipMemUnmap(p, bytes);
    hipMemAddressFree(p, bytes);
    hipMemRelease((hipMemGenericAllocationHandle_t)(uintptr_t)vmm);
}

extern "C" int mp2vg_reserve_slots(mp2vg_ctx_t* c, int32_t nslots) {
    if (!c || nslots <= 0) return MP2VG_E_INVALID;
    HIPCHK(hipSetDevice(c->cfg.device));
    if (nslots <= c->nslots) return MP2VG_OK;
    HIPCHK(hipStreamSynchronize(c->stream));
    if (!c->d_sink) {
        HIPCHK(hipMalloc((void**)&c->d_sink, kPoolPad));
        HIPCHK(hipMemsetAsync(c->d_sink, 0, kPoolPad, c->stream));
    }
    // The slots come in blocks of 16 (MP2VG_POOL_CHUNK; 0 = one block for all), each block its own
    // allocation (frames, then tiles), added as the pool grows (no copy).  One pool-sized
    // allocation lands, in some processes, where the anchors' tile stores run 10-20 % slower
    // (c2 334.8k vs 365.4k frames/s, same library and box); blocks of 16 slots measured 349.4k /
    // 349.6k against 322.8k / 322.8k for one block on a box where the single block was slow
    // (profiles/r4/README.md, placement).
    static const int chunk = getenv("MP2VG_POOL_CHUNK") ? std::max(0, atoi(getenv("MP2VG_POOL_CHUNK"))) : 16;
    if (chunk > 0) {
        // the new blocks are committed to the context only once every allocation has succeeded: a
        // failed reserve leaves the pool (chunks, fptr, tptr, nslots) as it was, and frees its blocks
        std::vector<uint8_t*> blocks;
        std::vector<size_t> bsz;
        std::vector<uint64_t> fp, tp, vh;
        auto fail = [&](hipError_t e) {
            for (size_t i = 0; i < blocks.size(); i++) pool_block_free(blocks[i], bsz[i], vh[i]);
            set_error(std::string("hipMalloc (frame pool block): ") + hipGetErrorString(e));
            return MP2VG_E_HIP;
        };
        for (int s0 = c->nslots; s0 < nslots; s0 += chunk) {
            const int k = std::min(chunk, nslots - s0);
            uint8_t *f = nullptr, *t = nullptr;
            size_t got = 0;
            uint64_t h = 0;
            hipError_t e = pool_block_alloc(c->cfg.device, c->slot_stride * k + kPoolPad, &f, &got, &h);
            if (e != hipSuccess) return fail(e);
            blocks.push_back(f);
            bsz.push_back(got);
            vh.push_back(h);
            if ((e = pool_block_alloc(c->cfg.device, c->tile_stride * k, &t, &got, &h)) != hipSuccess) return fail(e);
            blocks.push_back(t);
            bsz.push_back(got);
            vh.push_back(h);
            if ((e = hipMemsetAsync(f, 0, c->slot_stride * k + kPoolPad, c->stream)) != hipSuccess ||
                (e = hipMemsetAsync(t, 0, c->tile_stride * k, c->stream)) != hipSuccess)
                return fail(e);
            for (int i = 0; i < k; i++) {
                fp.push_back((uint64_t)(uintptr_t)(f + (size_t)i * c->slot_stride));
                tp.push_back((uint64_t)(uintptr_t)(t + (size_t)i * c->tile_stride));
            }
        }
        c->chunks.insert(c->chunks.end(), blocks.begin(), blocks.end());
        c->chunk_bytes.insert(c->chunk_bytes.end(), bsz.begin(), bsz.end());
        c->chunk_vmm.insert(c->chunk_vmm.end(), vh.begin(), vh.end());
        c->fptr.insert(c->fptr.end(), fp.begin(), fp.end());
        c->tptr.insert(c->tptr.end(), tp.begin(), tp.end());
        return finish_reserve(c, nslots);
    }
    uint8_t* p = nullptr;
    uint8_t* t = nullptr;
    size_t bytes = c->slot_stride * nslots + kPoolPad;
    const size_t tbytes = c->tile_stride * nslots;
#ifdef MP2VG_DEV_ABLATIONS
    // dev knob for the pool-placement study (profiles/r4/README.md): 1 = physically contiguous
    // (hipDeviceMallocContiguous, default allocation if the driver refuses it); 5 = the process's
    // first block (pool-sized, or MP2VG_BALLAST_MB) is held for good.  Dev builds only.
    static const int pool_alloc = getenv("MP2VG_POOL_ALLOC") ? atoi(getenv("MP2VG_POOL_ALLOC")) : 0;
    if (pool_alloc == 1 && hipExtMallocWithFlags((void**)&p, bytes, hipDeviceMallocContiguous) != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
    }
    static uint8_t* ballast = nullptr;
    static const size_t ballast_mb = getenv("MP2VG_BALLAST_MB") ? (size_t)atoll(getenv("MP2VG_BALLAST_MB")) : 0;
    if (pool_alloc == 5 && !ballast &&
        hipMalloc((void**)&ballast, ballast_mb ? ballast_mb << 20 : bytes + tbytes) != hipSuccess)
        (void)hipGetLastError(), ballast = nullptr;
#endif
    if (!p) HIPCHK(hipMalloc((void**)&p, bytes));
    if (hipMalloc((void**)&t, tbytes) != hipSuccess) {
        hipFree(p);
        set_error("out of device memory for the anchor tiles");
        return MP2VG_E_HIP;
    }
    HIPCHK(hipMemsetAsync(p, 0, bytes, c->stream));
    HIPCHK(hipMemsetAsync(t, 0, tbytes, c->stream));  // a never-decoded reference reads zeros, as its slot
    if (c->d_pool) {
        HIPCHK(hipMemcpyAsync(p, c->d_pool, c->slot_stride * c->nslots, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(t, c->d_tiles, c->tile_stride * c->nslots, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        HIPCHK(hipFree(c->d_pool));
        HIPCHK(hipFree(c->d_tiles));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    c->d_pool = p;
    c->d_tiles = t;
    c->fptr.resize(nslots);
    c->tptr.resize(nslots);
    for (int i = 0; i < nslots; i++) {
        c->fptr[i] = (uint64_t)(uintptr_t)(p + (size_t)i * c->slot_stride);
        c->tptr[i] = (uint64_t)(uintptr_t)(t + (size_t)i * c->tile_stride);
    }
    return finish_reserve(c, nslots);
}

// Validate the batch so no kernel access can leave its buffers, and compute dependency levels.
static int plan_batch(mp2vg_ctx_t* c, const mp2vg_picture_t* pics, int32_t npics, const mp2vg_mb_t* mbs,
                      uint64_t nmbs, const uint32_t* coefs, uint64_t ncoefs, std::vector<SliceDesc>& slices,
                      std::vector<Launch>& launches, std::vector<std::vector<int32_t>>* foot = nullptr,
                      bool trusted = false, TilePlan* tplan = nullptr) {
    const int mbw = c->cfg.width / 16, mbh = c->cfg.height / 16;
    const int nb = c->g.nblocks;
    // the I kernels address coefficient words with 32-bit byte offsets (a buffer resource)
    if (ncoefs + kCoefPad >= (1ull << 30)) {
        set_error("batch with 2^30 or more coefficient words (4 GB): split it");
        return MP2VG_E_INVALID;
    }
    std::vector<int> level(npics, 0);
    std::vector<int> last_write(c->nslots, -1), max_read(c->nslots, -1);
    int maxlevel = -1;
    // per-picture record validation (O(MBs + coefficient words)) runs on host threads; the first
    // failing picture in batch order reports its error
    std::vector<uint8_t> uses_of(2 * (size_t)npics, 0);
    std::vector<const char*> err(npics, nullptr);
    // records of this library's own parser (the drop-in decoder) meet the contract by
    // construction (tests/test_validate.py: parsed batches validate): only the picture-level checks
    // and the reference usage the scheduler needs are computed for them
    // the picture type picks the kernel mode of its launch and whether it stores anchor tiles
    // (TilePlan): only 1 (I), 2 (P) and 3 (B) exist (mp2vg.h)
    auto bad_type = [&](int p) { return pics[p].picture_coding_type < 1 || pics[p].picture_coding_type > 3; };
    auto uses_only = [&](int p) -> const char* {
        const mp2vg_picture_t& P = pics[p];
        if (bad_type(p)) return "picture_coding_type is not 1 (I), 2 (P) or 3 (B)";
        if (P.mb_width != mbw || P.mb_height != mbh) return "picture size differs from the context geometry";
        if (P.dst_slot < 0 || P.dst_slot >= c->nslots || P.fwd_slot >= c->nslots || P.bwd_slot >= c->nslots)
            return "frame slot out of range (mp2vg_reserve_slots)";
        const uint64_t nm = (uint64_t)mbw * mbh;
        if ((uint64_t)P.mb_first + nm > nmbs) return "picture MB range outside the batch";
        bool uses[2] = {false, false};
        for (uint64_t k = 0; k < nm; k++) {
            const mp2vg_mb_t& m = mbs[P.mb_first + k];
            // the one O(MB) check kept on the trusted path: the kernel's coefficient loads of a
            // P/B group are raw pointers, so a word range past the batch would read out of bounds
            if ((uint64_t)m.coef_off + m.ncoef > ncoefs) return "MB coefficient range outside the batch";
            const uint16_t f = m.flags;
            if (!(f & MP2VG_MB_INTRA)) {
                uses[0] |= (f & MP2VG_MB_FWD) || !(f & MP2VG_MB_BWD);
                uses[1] |= (f & MP2VG_MB_BWD) != 0;
            }
        }
        uses_of[2 * (size_t)p] = uses[0];
        uses_of[2 * (size_t)p + 1] = uses[1];
        return nullptr;
    };
    auto validate = [&](int p) -> const char* {
        if (trusted) return uses_only(p);
        const mp2vg_picture_t& P = pics[p];
        if (bad_type(p)) return "picture_coding_type is not 1 (I), 2 (P) or 3 (B)";
        if (P.mb_width != mbw || P.mb_height != mbh) return "picture size differs from the context geometry";
        if (P.dst_slot < 0 || P.dst_slot >= c->nslots || P.fwd_slot >= c->nslots || P.bwd_slot >= c->nslots)
            return "frame slot out of range (mp2vg_reserve_slots)";
        const uint64_t nm = (uint64_t)mbw * mbh;
        if ((uint64_t)P.mb_first + nm > nmbs) return "picture MB range outside the batch";
        bool uses[2] = {false, false};
        for (uint64_t k = 0; k < nm; k++) {
            const mp2vg_mb_t& m = mbs[P.mb_first + k];
            if (m.x != k % mbw || m.y != k / mbw) return "MB records not in raster order";
            if ((uint64_t)m.coef_off + m.ncoef > ncoefs) return "MB coefficient range outside the batch";
            // the kernel takes a word's MB (inside its 4-MB group) from bits 26-27, and files DC /
            // '1s' words under the block position of i, which must be 0
            const uint32_t tag = MP2VG_COEF_MBX(m.x);
            const uint32_t first = MP2VG_COEF_DC | MP2VG_COEF_FIRST1S;
            uint32_t bad = 0, blocks = 0, pos0 = 0;
            const uint32_t* w = coefs + m.coef_off;
            for (uint32_t j = 0; j < m.ncoef; j++) {
                bad |= (w[j] & 0x9C000000u) ^ tag;
                blocks |= 1u << MP2VG_COEF_BLOCK(w[j]);
                pos0 |= (w[j] & first) ? MP2VG_COEF_POS(w[j]) : 0u;
            }
            if (bad) return "coefficient word bits 26-28 are not the MB column mod 8 (or bit 31 is set)";
            if (pos0) return "DC or '1s' coefficient word with a nonzero scan position";
            // the kernel files a word under its block's coded-block slot: the block must be coded
            if (blocks & ~(uint32_t)m.cbp) return "coefficient word of a block the MB's cbp does not code";
            // the kernel streams the coefficient words of consecutive MBs of a row as one range
            if (k % mbw != 0) {
                const mp2vg_mb_t& pm = mbs[P.mb_first + k - 1];
                if ((uint64_t)pm.coef_off + pm.ncoef != m.coef_off)
                    return "coefficient words of a macroblock row are not contiguous";
            }
            if (m.cbp >> nb) return "cbp names a block the chroma format does not have";
            // 4:4:4 field DCT: the reference places blocks 10/11 at (dct_type ? 1 : 8) * stride + 8
            // with the doubled LUMA stride (mb_decoder.cpp:193-194), i.e. two rows down and one
            // row into the next MB row, leaving odd rows unwritten; the parser rejects such
            // streams, and no record producer may hand them to the kernel (spec placement)
            if (nb == 12 && (m.flags & MP2VG_MB_DCT_FIELD) && m.cbp)
                return "4:4:4 field-DCT macroblock (reference block 10/11 placement is unsupported)";
            // intra MBs code every block (the I kernel's 4:4:4 store writes clamp(residual) with
            // no prediction underneath), and the I kernel dequantises every word as intra
            if ((m.flags & MP2VG_MB_INTRA) && m.cbp != (1u << nb) - 1)
                return "intra macroblock whose cbp does not code every block";
            if (P.picture_coding_type == 1 && !(m.flags & MP2VG_MB_INTRA)) return "non-intra macroblock in an I picture";
            if (!(m.flags & MP2VG_MB_INTRA)) {
                const bool dir[2] = {(m.flags & MP2VG_MB_FWD) || !(m.flags & MP2VG_MB_BWD), (m.flags & MP2VG_MB_BWD) != 0};
                uses[0] |= dir[0];
                uses[1] |= dir[1];
                // every vector the kernel applies reads inside the reference planes (the input
                // contract the reference relies on, mb_decoder.cpp:212-289): the kernel's row
                // offsets are not clamped into the plane
                const bool field = m.flags & MP2VG_MB_FIELD_MC;
                for (int r = 0; r < (field ? 2 : 1); r++)
                    for (int s = 0; s < 2; s++)
                        if (dir[s] && !mc_reads_inside(c->g, m.x, m.y, m.mv[r][s][0], m.mv[r][s][1], field,
                                                       (m.flags & MP2VG_MB_FS_BIT(r, s)) ? 1 : 0, r))
                            return "motion vector reads outside the reference planes";
            }
        }
        uses_of[2 * (size_t)p] = uses[0];
        uses_of[2 * (size_t)p + 1] = uses[1];
        return nullptr;
    };
    parallel_for(npics, 16, [&](int p) { err[p] = validate(p); });
    for (int p = 0; p < npics; p++) {
        const mp2vg_picture_t& P = pics[p];
        if (err[p]) {
            set_error(err[p]);
            return MP2VG_E_INVALID;
        }
        const bool uses[2] = {uses_of[2 * (size_t)p] != 0, uses_of[2 * (size_t)p + 1] != 0};
        // the P loop predicts every non-intra MB from the forward reference (recon.hip issue_pass)
        if (P.picture_coding_type == 2 && uses[1]) {
            set_error("backward prediction in a P picture");
            return MP2VG_E_INVALID;
        }
        if ((uses[0] && P.fwd_slot < 0) || (uses[1] && P.bwd_slot < 0)) {
            set_error("picture predicts from a missing reference slot");
            return MP2VG_E_INVALID;
        }
        int lv = 0;
        if (uses[0]) lv = std::max(lv, last_write[P.fwd_slot] + 1);
        if (uses[1]) lv = std::max(lv, last_write[P.bwd_slot] + 1);
        lv = std::max(lv, last_write[P.dst_slot] + 1);  // WAW
        lv = std::max(lv, max_read[P.dst_slot] + 1);    // WAR
        if ((uses[0] && P.fwd_slot == P.dst_slot) || (uses[1] && P.bwd_slot == P.dst_slot)) {
            set_error("picture predicts from its own slot");
            return MP2VG_E_INVALID;
        }
        level[p] = lv;
        if (uses[0]) max_read[P.fwd_slot] = std::max(max_read[P.fwd_slot], lv);
        if (uses[1]) max_read[P.bwd_slot] = std::max(max_read[P.bwd_slot], lv);
        last_write[P.dst_slot] = lv;
        max_read[P.dst_slot] = -1;
        maxlevel = std::max(maxlevel, lv);
    }
    // one launch per dependency level.  A level of one picture type runs the kernel specialised --
    // and register-allocated -- for its motion-compensation mode: I (none), P (forward only), B
    // (both directions).  A level that mixes types (B pictures next to the following P anchor)
    // runs the mixed kernel, which picks the mode per workgroup from the picture type: one launch
    // tail per level instead of one per type.  Pictures stay in decode order, so every XCD's
    // contiguous share of the slices holds the same mix of P and B work.
    //
    // Independent picture sets run on separate streams: pictures that touch a common slot (as
    // destination or used reference) are one component; components (closed GOPs) are dealt to
    // c->nstreams sets, each with its own chain of level launches.  The streams run freely, so one
    // set's VALU-heavy I level overlaps another's memory-heavy B level and fills its launch tails.
    const int nsets = std::max(1, std::min(c->nstreams, npics));
    std::vector<int> parent(npics);
    for (int p = 0; p < npics; p++) parent[p] = p;
    auto find = [&](int x) {
        while (parent[x] != x) x = parent[x] = parent[parent[x]];
        return x;
    };
    {
        std::vector<int> owner(c->nslots, -1);
        for (int p = 0; p < npics; p++) {
            const mp2vg_picture_t& P = pics[p];
            const int sl[3] = {P.dst_slot, uses_of[2 * (size_t)p] ? P.fwd_slot : -1,
                               uses_of[2 * (size_t)p + 1] ? P.bwd_slot : -1};
            for (int s : sl) {
                if (s < 0) continue;
                if (owner[s] < 0) owner[s] = p;
                else parent[find(p)] = find(owner[s]);
            }
        }
    }
    std::vector<int> set_of(npics, 0), root_set(npics, -1);
    std::vector<size_t> load(nsets, 0);
    for (int p = 0; p < npics; p++) {  // components in decode order of their first picture
        const int r = find(p);
        if (root_set[r] < 0) root_set[r] = (int)(std::min_element(load.begin(), load.end()) - load.begin());
        set_of[p] = root_set[r];
        load[set_of[p]]++;
    }
    if (foot) {  // each set's slot footprint: the next batch's sets wait only for overlapping ones
        foot->assign(nsets, {});
        std::vector<int8_t> seen((size_t)c->nslots * nsets, 0);
        for (int p = 0; p < npics; p++) {
            const mp2vg_picture_t& P = pics[p];
            const int sl[3] = {P.dst_slot, uses_of[2 * (size_t)p] ? P.fwd_slot : -1,
                               uses_of[2 * (size_t)p + 1] ? P.bwd_slot : -1};
            for (int x : sl)
                if (x >= 0 && !seen[(size_t)set_of[p] * c->nslots + x]) {
                    seen[(size_t)set_of[p] * c->nslots + x] = 1;
                    (*foot)[set_of[p]].push_back(x);
                }
        }
    }
    // anchor tiles (TilePlan): which pictures store them, which slots the batch reads from earlier
    // batches, and the tiles state each written slot is left in
    std::vector<uint8_t> need(npics, 0);
    {
        std::vector<int> writer(c->nslots, -1);
        std::vector<uint8_t> ext(c->nslots, 0);
        for (int p = 0; p < npics; p++) {
            const mp2vg_picture_t& P = pics[p];
            const int rs[2] = {uses_of[2 * (size_t)p] ? P.fwd_slot : -1, uses_of[2 * (size_t)p + 1] ? P.bwd_slot : -1};
            for (int s : rs) {
                if (s < 0) continue;
                if (writer[s] >= 0) {
                    need[writer[s]] = 1;
                } else if (!ext[s]) {
                    ext[s] = 1;
                    if (tplan) tplan->ext_reads.push_back({s, set_of[p]});
                }
            }
            writer[P.dst_slot] = p;
        }
        for (int p = npics - 1, anchors = 0; p >= 0 && anchors < 2; p--)
            if (pics[p].picture_coding_type != 3) need[p] = 1, anchors++;
        if (tplan)
            for (int p = 0; p < npics; p++) tplan->writes.push_back({pics[p].dst_slot, need[p]});
    }
    slices.clear();
    launches.clear();
    // MB rows per slice: 1 (two slices per workgroup in P/B launches, `mates` below; before them
    // P/B workgroups took two rows of one picture: a 1080p row is 30 four-MB groups, 8/8/7/7 over
    // a workgroup's four waves, and two rows made it 15 per wave, +2.4 % over one row).  Groups
    // never straddle rows when the row is a multiple of 4 MBs; other widths keep 1 row and no
    // mates.  (MP2VG_SLICE_ROWS / MP2VG_SLICE_ROWS_I override in dev builds.)
    static const int rows_pb = dev_env("MP2VG_SLICE_ROWS") ? std::max(1, atoi(dev_env("MP2VG_SLICE_ROWS"))) : 2;
    // P/B launches run one-row slices, two per workgroup (`mates`, recon.hip recon_kernel): the
    // consecutive slices of a reference-sharing cluster, i.e. the same MB row of two pictures that
    // read the same anchors, waves 0-1 on one and 2-3 on the other.  Same balance as two rows of
    // one picture (15 groups per wave), half the MB rows in flight per XCD, and both pictures'
    // taps of one anchor region on one CU: c2 +0.9 %, c3 +1.9 % over two-row slices (same box,
    // profiles/r5/README.md).  (MP2VG_MATES=0 in dev builds: two-row slices.)
    static const int mates = !dev_env("MP2VG_MATES") ? 2 : atoi(dev_env("MP2VG_MATES")) == 4 ? 4 : (atoi(dev_env("MP2VG_MATES")) ? 2 : 0);
    // An odd cluster's two-reference pictures are mates row by row and its one-reference picture
    // is its own mate (two consecutive rows): one-stream c2 span -0.8 to -1.5 %, the P / one-
    // direction B level launch -1.5 to -2.3 % (same box, profiles/r5/README.md).  (MP2VG_PAIR_ORDER=0
    // in dev builds: plain row-by-row interleave.)
    static const bool pair_order = !dev_env("MP2VG_PAIR_ORDER") || atoi(dev_env("MP2VG_PAIR_ORDER")) != 0;
    // I-only launches: one row per slice, two in 4:4:4 (its heavy I groups -- 12 blocks, four
    // workgroups per CU -- pack the two picture sets' concurrent launches better with half as many,
    // longer workgroups: c5 +1.8 to +6.7 %, three same-box rounds; c1 (4:2:0) no gain)
    static const int rows_i_env = dev_env("MP2VG_SLICE_ROWS_I") ? std::max(1, atoi(dev_env("MP2VG_SLICE_ROWS_I"))) : 0;
    const int rows_i = rows_i_env ? rows_i_env : (c->g.cf == 3 ? 2 : 1);
    static const int i_split = dev_env("MP2VG_I_SPLIT") ? std::max(1, atoi(dev_env("MP2VG_I_SPLIT"))) : 1;
    static const int i_mbs = dev_env("MP2VG_I_SLICE_MBS") ? std::max(0, atoi(dev_env("MP2VG_I_SLICE_MBS"))) : 0;
    // I launches fill whole rounds of resident workgroups: the default slice (rows_i rows), or up
    // to a quarter more 4-MB groups cut across rows, whichever leaves the launch's last round of
    // workgroups least empty, against the device's CUs x the I kernel's workgroups per CU (6, or 4
    // in 4:4:4) shared by the picture sets' concurrent I launches.  (c1: 128-MB slices, 4.98
    // instead of 5.31 rounds; c5: 256-MB slices, 1.99 instead of 2.13; one-stream I launch -1.5 %
    // and -3.6 %, profiles/r6/README.md §10.)  A gain under 0.1 round keeps the default.
    auto i_slice_groups = [&](size_t npic_launch) -> int {
        const int s0 = rows_i * mbw / 4;
        if (rows_i_env || i_mbs || i_split > 1 || mbw % 4) return s0;
        const double cap = (double)(c->ncu > 0 ? c->ncu : 256) * (c->g.cf == 3 ? 4 : 6) / std::max(1, nsets);
        const double gtot = (double)npic_launch * (mbw / 4) * mbh;
        auto waste = [&](int sg) {
            const double r = std::ceil(gtot / sg) / cap;
            return std::ceil(r) - r;
        };
        int best = s0;
        for (int sg = s0 + 1; sg <= s0 + s0 / 4; sg++)
            if (waste(sg) < waste(best)) best = sg;
        return waste(s0) - waste(best) >= 0.1 ? best : s0;
    };
    for (int set = 0; set < nsets; set++)
    for (int q = 0; q <= maxlevel; q++) {
        std::vector<int> lp;
        for (int p = 0; p < npics; p++)
            if (level[p] == q && set_of[p] == set) lp.push_back(p);
        if (lp.empty()) continue;
        Launch l;
        l.begin = (uint32_t)slices.size();
        // B pictures that predict in one direction only (a closed GOP's leading B pictures:
        // backward only) run the one-reference P loop with that reference (SliceDesc.reserved
        // bits 1-2, recon.hip issue_pass): a launch of P and such B pictures is a P launch
        // (MP2VG_ONE_DIR_B=0 in dev builds: every B picture in the B loop)
        static const bool route = !dev_env("MP2VG_ONE_DIR_B") || atoi(dev_env("MP2VG_ONE_DIR_B")) != 0;
        auto one_dir = [&](int p) {
            return route && pics[p].picture_coding_type == 3 && !(uses_of[2 * (size_t)p] && uses_of[2 * (size_t)p + 1]);
        };
        int types = 0;
        for (int p : lp) {
            const int pct = pics[p].picture_coding_type;
            types |= 1 << (pct == 1 ? 0 : (pct == 2 || one_dir(p) ? 1 : 2));
        }
        // Pictures that read a common reference slot (the two B pictures between a pair of
        // anchors and the P picture after them) form a cluster whose slices are interleaved row
        // by row, so their workgroups read the same reference lines at about the same time on
        // the same XCD (measured: +0.6 % on c2).
        auto reads = [&](int p, int s) { return s >= 0 && (pics[p].fwd_slot == s || pics[p].bwd_slot == s); };
        // bit 0: the picture stores its anchor tiles in the loop (I and P; B pictures read later
        // get theirs from tile_convert after the launch, TilePlan.post); bit 1: one-direction B
        // picture (P loop); bit 2: its one direction is backward
        auto sflags = [&](int p) -> uint32_t {
            const bool b = pics[p].picture_coding_type == 3;
            const bool bwd_only = !uses_of[2 * (size_t)p] && uses_of[2 * (size_t)p + 1];
            return (uint32_t)(need[p] && !b) | (one_dir(p) ? 2u : 0u) | (one_dir(p) && bwd_only ? 4u : 0u);
        };
        size_t i = 0;
        while (i < lp.size()) {
            size_t j = i + 1;
            while (j < lp.size() && j - i < 4) {
                bool share = false;
                for (size_t k = i; k < j && !share; k++)
                    share = reads(lp[j], pics[lp[k]].fwd_slot) || reads(lp[j], pics[lp[k]].bwd_slot);
                if (!share) break;
                j++;
            }
            const int slice_rows = (mbw % 4 != 0) ? 1 : (types == 1 ? rows_i : (mates ? 1 : rows_pb));
            auto push = [&](size_t k, int r) {
                slices.push_back({(uint32_t)lp[k], pics[lp[k]].mb_first + (uint32_t)(r * mbw),
                                  (uint32_t)(std::min(slice_rows, mbh - r) * mbw), sflags(lp[k])});
            };
            const bool paired = pair_order && mates == 2 && types != 1 && mbw % 4 == 0;
            if (paired && (j - i) % 2 == 1 && j - i > 1) {
                // an odd cluster (the P picture and the two B pictures before it): the B pictures,
                // which share both references, are mates row by row, and the odd one (the
                // one-reference picture) is its own mate, two consecutive rows
                size_t o = j - 1;
                for (size_t k = i; k < j; k++)
                    if (pics[lp[k]].picture_coding_type == 2 || one_dir(lp[k])) o = k;
                for (int r = 0; r < mbh; r += 2) {
                    for (int rr = r; rr < std::min(r + 2, mbh); rr++)
                        for (size_t k = i; k < j; k++)
                            if (k != o) push(k, rr);
                    for (int rr = r; rr < std::min(r + 2, mbh); rr++) push(o, rr);
                }
            } else if (types == 1 && mbw % 4 == 0 &&
                       ((i_mbs > 0 && i_mbs % 4 == 0) || i_slice_groups(lp.size()) != rows_i * mbw / 4)) {
                // I slices of i_mbs MBs (a multiple of 4: groups never straddle rows; the dev
                // MP2VG_I_SLICE_MBS, else i_slice_groups), cut across rows, the picture's last
                // one shorter
                const int cut = i_mbs > 0 ? i_mbs : 4 * i_slice_groups(lp.size());
                const int total = mbw * mbh;
                for (int m0 = 0; m0 < total; m0 += cut)
                    for (size_t k = i; k < j; k++)
                        slices.push_back({(uint32_t)lp[k], pics[lp[k]].mb_first + (uint32_t)m0,
                                          (uint32_t)std::min(cut, total - m0), sflags(lp[k])});
            } else if (types == 1 && slice_rows == 1 && i_split > 1 && (mbw / i_split) % 4 == 0 && mbw % i_split == 0) {
                // (dev) I launches in pieces of a row: more, shorter workgroups for the launch tail
                const int pw = mbw / i_split;
                for (int r = 0; r < mbh; r++)
                    for (size_t k = i; k < j; k++)
                        for (int q = 0; q < i_split; q++)
                            slices.push_back({(uint32_t)lp[k], pics[lp[k]].mb_first + (uint32_t)(r * mbw + q * pw),
                                              (uint32_t)pw, sflags(lp[k])});
            } else {
                for (int r = 0; r < mbh; r += slice_rows)
                    for (size_t k = i; k < j; k++) push(k, r);
            }
            i = j;
        }
        l.end = (uint32_t)slices.size();
        l.mcm = types == 1 ? 0 : (types == 2 ? 1 : (types == 4 ? 2 : 3));
        // (dev) A 4:2:0 / 4:2:2 I-only launch in which at most a quarter of the pictures store tiles (an
        // I-only stream: the batch's last two pictures) runs the I kernel without the tile store
        // code (mode 4: 71 instead of 79 VGPRs, 7 waves per SIMD instead of 6; the 4:4:4 kernel
        // keeps its 4) and converts those pictures' tiles after it (tile_convert, same stream).
        // Measured neutral on c1 twice (one-stream I launch 0.286 ms either way, profiles/r5/README.md;
        // 388-419k against 402-419k frames/s, profiles/r6/ab_mode4_c1.txt): the skipped stores were
        // already branched over per slice.  So a dev switch only: MP2VG_I_TILEFREE=1 in dev builds
        // enables it, =2 runs it for every I-only launch, whatever stores tiles, 4:4:4 too.
        static const int tilefree = dev_env("MP2VG_I_TILEFREE") ? atoi(dev_env("MP2VG_I_TILEFREE")) : 0;
        int nneed = 0;
        for (int p : lp) nneed += need[p];
        if (types == 1 && (tilefree == 2 || (tilefree && c->g.cf != 3 && nneed * 4 <= (int)lp.size()))) {
            l.mcm = 4;
            for (uint32_t k = l.begin; k < l.end; k++) slices[k].reserved = 0;
        }
        l.level = q;
        l.set = set;
        // (4:4:4 kernels hold two slices' tables at most: Lds::NH)
        l.mates = (mates && types != 1 && l.mcm != 0 && l.mcm != 4 && mbw % 4 == 0) ? (c->g.cf == 3 ? std::min(mates, 2) : mates) : 0;
        if (tplan)
            for (int p : lp)
                if (need[p] && (pics[p].picture_coding_type == 3 || l.mcm == 4))
                    tplan->post.push_back({(int32_t)launches.size(), pics[p].dst_slot});
        launches.push_back(l);
    }
    return MP2VG_OK;
}

static int batch_upload(mp2vg_ctx_t* c, const mp2vg_picture_t* pics, int32_t npics, const mp2vg_mb_t* mbs,
                        uint64_t nmbs, const uint32_t* coefs, uint64_t ncoefs, bool pinned, bool async,
                        bool trusted = false) {
    if (!c || !pics || npics <= 0 || !mbs || (!coefs && ncoefs)) return MP2VG_E_INVALID;
    HIPCHK(hipSetDevice(c->cfg.device));
    c->batch_ready = false;
    std::vector<SliceDesc> slices;
    std::vector<Launch> lb;
    std::vector<std::vector<int32_t>> foot;
    TilePlan tplan;
    double tp = now_ms();
    int rc = plan_batch(c, pics, npics, mbs, nmbs, coefs, ncoefs, slices, lb, &foot, trusted, &tplan);
    if (rc != MP2VG_OK) return rc;
    tp = trace_phase("upload: plan", tp);
    // the other bank from the last upload; the decode queued on it is still allowed to run
    const int k = (c->cur + 1) & 1;
    Bank& b = c->bank[k];
    if (b.decoded) HIPCHK(hipEventSynchronize(b.consumed));
    if ((rc = grow(b.d_pics, b.cap_pics, (size_t)npics)) != MP2VG_OK) return rc;
    if ((rc = grow(b.d_mbs, b.cap_mbs, (size_t)nmbs + kMbPad)) != MP2VG_OK) return rc;
    // the kernel loads 128 words from the first coefficient of each MB group unconditionally
    if ((rc = grow(b.d_coefs, b.cap_coefs, (size_t)ncoefs + kCoefPad)) != MP2VG_OK) return rc;
    if ((rc = grow(b.d_slices, b.cap_slices, slices.size())) != MP2VG_OK) return rc;
    // the post-launch tile conversions' slot lists, grouped by launch
    std::vector<int32_t> ps;
    std::vector<std::pair<int32_t, int32_t>> post_of(lb.size(), {0, 0});
    for (size_t i = 0; i < lb.size(); i++) {
        post_of[i].first = (int32_t)ps.size();
        for (const auto& pc : tplan.post)
            if (pc.first == (int32_t)i) ps.push_back(pc.second);
        post_of[i].second = (int32_t)ps.size();
    }
    if (!ps.empty() && (rc = grow(b.d_post, b.cap_post, ps.size())) != MP2VG_OK) return rc;
    const size_t pic_bytes = sizeof(mp2vg_picture_t) * npics, sl_bytes = sizeof(SliceDesc) * slices.size(),
                 ps_bytes = sizeof(int32_t) * ps.size();
    if (async) {
        // the drop-in's asynchronous upload: the small arrays go through the bank's own pinned
        // staging block, with no host wait (a synchronised staged copy would wait for the previous
        // chunk's record copies: the chunk loop then ran at the H2D rate, 0.6 ms per 16 frames).
        // The block's previous copies finished before the bank's previous decode, waited for above.
        HIPCHK(hipEventSynchronize(b.uploaded));
        const size_t o1 = (pic_bytes + 255) & ~(size_t)255, o2 = o1 + ((sl_bytes + 255) & ~(size_t)255);
        const size_t need = o2 + ps_bytes;
        if (need > b.cap_small) {
            if (b.h_small) HIPCHK(hipHostFree(b.h_small));
            b.h_small = nullptr;
            b.cap_small = 0;
            const size_t cap = std::max(need, (size_t)1 << 20);
            HIPCHK(hipHostMalloc((void**)&b.h_small, cap, hipHostMallocDefault));
            b.cap_small = cap;
        }
        memcpy(b.h_small, pics, pic_bytes);
        memcpy(b.h_small + o1, slices.data(), sl_bytes);
        if (ps_bytes) memcpy(b.h_small + o2, ps.data(), ps_bytes);
        HIPCHK(hipMemcpyAsync(b.d_pics, b.h_small, pic_bytes, hipMemcpyHostToDevice, c->ustream));
        HIPCHK(hipMemcpyAsync(b.d_slices, b.h_small + o1, sl_bytes, hipMemcpyHostToDevice, c->ustream));
        if (ps_bytes) HIPCHK(hipMemcpyAsync(b.d_post, b.h_small + o2, ps_bytes, hipMemcpyHostToDevice, c->ustream));
    } else {
        // picture records (small, may sit in pageable memory either way), this function's own
        // slice descriptors and post lists go through staging first: the staged copies end
        // synchronised
        if ((rc = upload(c, b.d_pics, pics, pic_bytes, false)) != MP2VG_OK) return rc;
        if ((rc = upload(c, b.d_slices, slices.data(), sl_bytes, false)) != MP2VG_OK) return rc;
        if (ps_bytes && (rc = upload(c, b.d_post, ps.data(), ps_bytes, false)) != MP2VG_OK) return rc;
    }
    if ((rc = upload(c, b.d_mbs, mbs, sizeof(mp2vg_mb_t) * nmbs, pinned)) != MP2VG_OK) return rc;
    if (ncoefs && (rc = upload(c, b.d_coefs, coefs, sizeof(uint32_t) * ncoefs, pinned)) != MP2VG_OK) return rc;
    HIPCHK(hipEventRecord(b.uploaded, c->ustream));
    // the caller's host buffers are free again, unless it asked for an asynchronous upload of
    // pinned buffers (it then waits with ctx_wait_upload before rewriting them)
    if (!async) HIPCHK(hipStreamSynchronize(c->ustream));
    trace_phase("upload: copy", tp);
    b.launches = std::move(lb);
    b.foot = std::move(foot);
    b.post_of = std::move(post_of);
    b.tiles = std::move(tplan);
    b.npics = npics;
    c->cur = k;
    c->batch_ready = true;
    return MP2VG_OK;
}

extern "C" int mp2vg_batch_validate(const mp2vg_config_t* cfg, int32_t nslots, const mp2vg_picture_t* pics,
                                    int32_t npics, const mp2vg_mb_t* mbs, uint64_t nmbs, const uint32_t* coefs,
                                    uint64_t ncoefs, int32_t* nlaunches, int32_t* launch_of_pic,
                                    int32_t* launch_mode, int32_t max_launches) {
    if (!cfg || nslots <= 0 || !pics || npics <= 0 || !mbs || (!coefs && ncoefs)) return MP2VG_E_INVALID;
    if (mp2vg_frame_geometry(cfg, nullptr, nullptr, nullptr, nullptr) != MP2VG_OK) return MP2VG_E_INVALID;
    // a host-side shell of a context: plan_batch reads only the geometry and the slot count
    mp2vg_ctx_t shell;
    shell.cfg = *cfg;
    shell.g.init(cfg->width, cfg->height, cfg->chroma_format);
    shell.nslots = nslots;
    shell.nstreams = default_streams(cfg);
    std::vector<SliceDesc> slices;
    std::vector<Launch> lb;
    const int rc = plan_batch(&shell, pics, npics, mbs, nmbs, coefs, ncoefs, slices, lb);
    if (rc != MP2VG_OK) return rc;
    if (nlaunches) *nlaunches = (int32_t)lb.size();
    for (size_t i = 0; i < lb.size(); i++) {
        if (launch_mode && (int32_t)i < max_launches) launch_mode[i] = lb[i].mcm;
        for (uint32_t k = lb[i].begin; launch_of_pic && k < lb[i].end; k++) launch_of_pic[slices[k].pic] = (int32_t)i;
    }
    return MP2VG_OK;
}

extern "C" int mp2vg_batch_upload(mp2vg_ctx_t* c, const mp2vg_picture_t* pics, int32_t npics,
                                  const mp2vg_mb_t* mbs, uint64_t nmbs, const uint32_t* coefs,
                                  uint64_t ncoefs) {
    return batch_upload(c, pics, npics, mbs, nmbs, coefs, ncoefs, false, false);
}

namespace mp2vg {
// Drop-in decoder (decoder.cpp): records in pinned host memory go to the device without staging
// and without waiting for the copies.  Its pinned buffer set i feeds bank i (banks alternate per
// upload): before rewriting set ctx_next_bank(), it calls ctx_wait_upload(ctx, that bank).  The
// records come from this library's parser, so the per-macroblock validation is skipped (trusted).
int batch_upload_pinned(mp2vg_ctx_t* c, const mp2vg_picture_t* pics, int32_t npics, const mp2vg_mb_t* mbs,
                        uint64_t nmbs, const uint32_t* coefs, uint64_t ncoefs) {
    return batch_upload(c, pics, npics, mbs, nmbs, coefs, ncoefs, true, true, true);
}
int ctx_next_bank(const mp2vg_ctx_t* c) { return (c->cur + 1) & 1; }
int ctx_wait_upload(mp2vg_ctx_t* c, int bank) {
    HIPCHK(hipEventSynchronize(c->bank[bank].uploaded));
    return MP2VG_OK;
}
hipStream_t ctx_stream(mp2vg_ctx_t* c) { return c->stream; }
void ctx_set_launch_timing(mp2vg_ctx_t* c, bool on) { c->launch_timing = on; }
}  // namespace mp2vg

static int batch_decode(mp2vg_ctx_t* c);

// ---- pool placement calibration ------------------------------------------------------------
// Identical contexts in one process decode the same batch up to 13 % apart, each keeping its
// speed, and which one is slow is not predicted by any per-block or pool-wide bandwidth probe
// (profiles/r6/README.md §8).  So a large pool measures its own placement once: at its first
// batch, the pool is copied into MP2VG_PLACE_CANDIDATES - 1 freshly allocated pools (same block
// sizes), the batch is decoded on each from the same starting state, and the pool with the
// shortest batch is kept (the others are freed).  Every candidate ends in the same state (the
// batch decoded), so the choice changes no output.
struct PoolSet {
    std::vector<uint8_t*> chunks;
    std::vector<size_t> bytes;
    std::vector<uint64_t> vmm, fptr, tptr;
};

static void pool_set_free(PoolSet& p) {
    for (size_t i = 0; i < p.chunks.size(); i++) pool_block_free(p.chunks[i], p.bytes[i], p.vmm[i]);
    p = PoolSet();
}

static void free_held_pools(mp2vg_ctx_t* c) {
    for (PoolSet* p : c->place_held) {
        pool_set_free(*p);
        delete p;
    }
    c->place_held.clear();
}

static PoolSet pool_take(mp2vg_ctx_t* c) {
    PoolSet p;
    p.chunks.swap(c->chunks);
    p.bytes.swap(c->chunk_bytes);
    p.vmm.swap(c->chunk_vmm);
    p.fptr.swap(c->fptr);
    p.tptr.swap(c->tptr);
    return p;
}

static hipError_t pool_install(mp2vg_ctx_t* c, PoolSet& p) {
    c->chunks.swap(p.chunks);
    c->chunk_bytes.swap(p.bytes);
    c->chunk_vmm.swap(p.vmm);
    c->fptr.swap(p.fptr);
    c->tptr.swap(p.tptr);
    p = PoolSet();
    hipError_t e = hipMemcpyAsync(c->d_tab, c->fptr.data(), sizeof(uint64_t) * c->nslots, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(c->d_tab + c->nslots, c->tptr.data(), sizeof(uint64_t) * c->nslots, hipMemcpyHostToDevice,
                           c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    return e;
}

// a copy of pool `src` (blocks of the same sizes, contents copied, slot addresses rebased)
static hipError_t pool_clone(mp2vg_ctx_t* c, const PoolSet& src, PoolSet& dst) {
    for (size_t i = 0; i < src.chunks.size(); i++) {
        uint8_t* q = nullptr;
        size_t got = 0;
        uint64_t h = 0;
        hipError_t e = pool_block_alloc(c->cfg.device, src.bytes[i], &q, &got, &h);
        if (e != hipSuccess) {
            pool_set_free(dst);
            return e;
        }
        dst.chunks.push_back(q);
        dst.bytes.push_back(got);
        dst.vmm.push_back(h);
        if ((e = hipMemcpyAsync(q, src.chunks[i], src.bytes[i], hipMemcpyDeviceToDevice, c->stream)) != hipSuccess) {
            pool_set_free(dst);
            return e;
        }
    }
    // blocks sorted by address, to map each slot pointer to its block
    std::vector<std::pair<uintptr_t, size_t>> order(src.chunks.size());
    for (size_t i = 0; i < order.size(); i++) order[i] = {(uintptr_t)src.chunks[i], i};
    std::sort(order.begin(), order.end());
    auto rebase = [&](uint64_t ptr) -> uint64_t {
        auto it = std::upper_bound(order.begin(), order.end(), std::make_pair((uintptr_t)ptr, (size_t)-1));
        const size_t i = std::prev(it)->second;
        return (uint64_t)(uintptr_t)dst.chunks[i] + (ptr - (uint64_t)(uintptr_t)src.chunks[i]);
    };
    for (uint64_t f : src.fptr) dst.fptr.push_back(rebase(f));
    for (uint64_t t : src.tptr) dst.tptr.push_back(rebase(t));
    return hipStreamSynchronize(c->stream);
}

// MP2VG_PLACE_CANDIDATES (pools tried, 1 = off; default 3, at most 6), MP2VG_PLACE_MIN_MB (smallest pool
// calibrated; default 4096), MP2VG_PLACE_ONE_STREAM=0 (multi-stream contexts only)
static int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}

// returns 1 when it did not run (the caller decodes), else the status of the calibrated decode.
// The batch is decoded 2 + 2 x candidates times: twice on the first pool (the GPU's clocks ramp
// over the first tens of ms of work: first-round times fall pool after pool whatever the pool),
// then twice on every candidate, round-robin, each candidate's time its faster run.  Decoding a
// batch again from its own output is exact only when no slot it writes is one it reads from
// before the batch (TilePlan.ext_reads); other batches are decoded once, uncalibrated.
static int calibrate_placement(mp2vg_ctx_t* c) {
    if (c->placed) return 1;
    const int k = std::max(1, std::min(6, env_int("MP2VG_PLACE_CANDIDATES", 3)));
    size_t pool = 0;
    for (size_t b : c->chunk_bytes) pool += b;
    if (k < 2 || c->chunks.empty() || pool < ((size_t)std::max(0, env_int("MP2VG_PLACE_MIN_MB", 4096)) << 20)) return 1;
    if (c->nstreams == 1 && !env_int("MP2VG_PLACE_ONE_STREAM", 1)) return 1;
    const Bank& bk = c->bank[c->cur];
    std::vector<uint8_t> written(c->nslots, 0);
    for (const auto& w : bk.tiles.writes)
        if (w.first >= 0 && w.first < c->nslots) written[w.first] = 1;
    for (const auto& r : bk.tiles.ext_reads)
        if (r.first >= 0 && r.first < c->nslots && written[r.first]) return 1;
    c->placed = true;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return 1;
    HIPCHK(hipStreamSynchronize(c->stream));
    std::vector<PoolSet> cand;
    cand.push_back(pool_take(c));
    // candidates only while an eighth of the device (at least 8 GB) stays free beside them, so
    // that the ones not kept can be held (below)
    const size_t reserve = std::max(total_b / 8, (size_t)8 << 30);
    for (int i = 1; i < k && free_b >= (size_t)i * pool + reserve; i++) {
        PoolSet p;
        if (pool_clone(c, cand[0], p) != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        cand.push_back(std::move(p));
    }
    const size_t n = cand.size();
    std::vector<float> ms(2 * n, 0.f);
    int rc = MP2VG_OK;
    auto run = [&](size_t i, float* t) -> int {
        if (pool_install(c, cand[i]) != hipSuccess) {
            cand[i] = pool_take(c);  // (the pool goes back to its candidate slot either way)
            return (int)MP2VG_E_HIP;
        }
        c->last_foot.clear();  // c->stream joined every set (synchronised by pool_install)
        int r = batch_decode(c);
        if (r == MP2VG_OK && t) r = mp2vg_batch_times(c, 0, t, nullptr, 0, nullptr);
        cand[i] = pool_take(c);
        return r;
    };
    const std::vector<uint8_t> tiles0 = c->tiles_ok;
    for (int w = 0; w < 2 && rc == MP2VG_OK; w++) rc = run(0, nullptr);  // warm-up
    for (int r = 0; r < 2 && rc == MP2VG_OK; r++)
        for (size_t i = 0; i < n && rc == MP2VG_OK; i++) {
            if (r == 0 && i > 0) c->tiles_ok = tiles0;  // a candidate's first decode starts from the batch's entry state
            rc = run(i, &ms[r * n + i]);
        }
    size_t best = 0;
    if (rc == MP2VG_OK)
        for (size_t i = 1; i < n; i++)
            if (std::min(ms[i], ms[n + i]) < std::min(ms[best], ms[n + best])) best = i;
    // The candidates not kept stay allocated until the context is destroyed: freeing them made
    // the kept pool's later batches 8 % slower for good (one-stream c2: 8.67-8.70 ms per batch
    // after the calibration measured it at 7.9-8.0, and still after a 10-s pause; held: 7.97; the
    // bench step: freed 380.7-383.3k, held 389.7-391.7k, uncalibrated 387.9-388.0k frames/s,
    // profiles/r6/README.md §11).  Held while an eighth of the device stays free (c3's bench holds
    // both its contexts' candidates: 231 of 288 GB; MP2VG_PLACE_HOLD=0 frees them, =1 holds them
    // regardless).
    size_t free_now = 0, total_now = 0;
    const bool room = hipMemGetInfo(&free_now, &total_now) == hipSuccess && free_now >= total_now / 8;
    const int hold_env = env_int("MP2VG_PLACE_HOLD", -1);
    const bool hold = hold_env < 0 ? room : hold_env != 0;
    for (size_t i = 0; i < n; i++)
        if (i != best && rc == MP2VG_OK) {
            if (hold)
                c->place_held.push_back(new PoolSet(std::move(cand[i])));
            else
                pool_set_free(cand[i]);
        }
    if (rc != MP2VG_OK) {  // an error keeps the original pool (its batch status is returned)
        for (size_t i = 1; i < n; i++) pool_set_free(cand[i]);
        best = 0;
    }
    HIPCHK(pool_install(c, cand[best]));
    c->place_ms = ms;
    c->place_kept = rc == MP2VG_OK ? (int)best : -1;
    if (getenv("MP2VG_TRACE")) {
        fprintf(stderr, "[mp2vg] placement: %zu candidate pools (others %s), batch ms (two rounds)", n,
                hold ? "held" : "freed");
        for (float m : ms) fprintf(stderr, " %.3f", m);
        fprintf(stderr, ", kept %zu\n", best);
    }
    return rc;
}

extern "C" int mp2vg_batch_decode(mp2vg_ctx_t* c) {
    if (!c) return MP2VG_E_INVALID;
    if (!c->batch_ready) {
        set_error("no batch uploaded");
        return MP2VG_E_STATE;
    }
    HIPCHK(hipSetDevice(c->cfg.device));
    const int rc = calibrate_placement(c);
    return rc == 1 ? batch_decode(c) : rc;
}

static int batch_decode(mp2vg_ctx_t* c) {
    Bank& b = c->bank[c->cur];
    const std::vector<Launch>& launches = b.launches;
    int nl = (int)launches.size();
    mp2vg_ctx::BatchEv& H = c->hist[c->seq % mp2vg_ctx::kHist];
    for (auto& e : H.b)
        if (!e) HIPCHK(hipEventCreate(&e));
    while (c->launch_timing && (int)H.l.size() < 2 * nl) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        H.l.push_back(e);
    }

    KArgs a;
    memset(&a, 0, sizeof a);
    a.pics = b.d_pics;
    a.mbs = b.d_mbs;
    a.coefs = b.d_coefs;
    a.slices = b.d_slices;
    a.sink = c->d_sink + kSinkOff;
    a.ftab = c->d_tab;
    a.ttab = c->d_tab + c->nslots;
    a.slot_bytes = c->g.slot_bytes;
    for (int i = 0; i < 3; i++) {
        a.plane_off[i] = c->g.plane_off[i];
        a.stride[i] = c->g.stride[i];
        a.ph[i] = c->g.ph[i];
    }
    // Each picture set's level launches run back to back on its own stream.  A set starts once
    // its records have landed and the sets of the previous batch that touched any of its slots
    // (as destination or used reference) are done -- not after the whole previous batch, so
    // back-to-back batches overlap set by set and one set's launch tails fill with the other's
    // work across batch boundaries too.  c->stream joins every set at the end, so API calls that
    // synchronise on it see the whole batch (they all do before touching slots).
    int nsets = 1;
    for (const Launch& L : launches) nsets = std::max(nsets, L.set + 1);
    while ((int)c->sstreams.size() < nsets) {
        hipStream_t st;
        hipEvent_t e;
        HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->sstreams.push_back(st);
        c->sev.push_back(e);
    }
    auto stream_of = [&](int set) { return c->sstreams[set]; };
    for (int set = 0; set < nsets; set++) {
        const hipStream_t st = stream_of(set);
        HIPCHK(hipStreamWaitEvent(st, b.uploaded, 0));
        for (int t = 0; t < (int)c->last_foot.size(); t++) {
            bool overlap = set >= (int)b.foot.size();  // no footprint: wait for everything
            for (size_t i = 0; !overlap && i < b.foot[set].size(); i++) overlap = c->last_foot[t][b.foot[set][i]];
            if (overlap) HIPCHK(hipStreamWaitEvent(st, c->sev[t], 0));
        }
    }
    // stale anchor tiles of slots this batch reads from earlier batches (rare: an MPEG-2 stream's
    // references are anchors, which store their tiles), rebuilt on the reading set's stream
    for (const auto& r : b.tiles.ext_reads)
        if (r.first < c->nslots && !c->tiles_ok[r.first]) {
            const int set = std::min(r.second, nsets - 1);
            HIPCHK(launch_tile_convert(a, c->g.cf, nullptr, 0, r.first, stream_of(set)));
            c->tiles_ok[r.first] = 1;
        }
    for (const auto& w : b.tiles.writes) c->tiles_ok[w.first] = w.second;
    // every set's start (after its waits): a set with no overlap with the previous batch starts
    // before set 0 does, so one start event on set 0 would under-report the batch span
    while ((int)H.s.size() < nsets) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        H.s.push_back(e);
    }
    for (int set = 0; set < nsets; set++) HIPCHK(hipEventRecord(H.s[set], stream_of(set)));
    H.ns = nsets;
    // launches are enqueued position by position across the sets (launch k of every set before
    // launch k + 1 of any), so a coupling wait always names an event already recorded this batch
    static const int couple = set_coupling();
    std::vector<int> pos(nl), at;  // position of launch i in its set's chain; (set, position) -> i
    std::vector<int> nper(nsets, 0);
    for (int i = 0; i < nl; i++) pos[i] = nper[launches[i].set]++;
    const int maxpos = *std::max_element(nper.begin(), nper.end());
    at.assign((size_t)nsets * maxpos, -1);
    for (int i = 0; i < nl; i++) at[(size_t)launches[i].set * maxpos + pos[i]] = i;
    if (couple && nsets > 1)
        while ((int)c->lev.size() < nl) {
            hipEvent_t e;
            HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            c->lev.push_back(e);
        }
    auto launch_at = [&](int set, int k) { return k >= 0 && k < nper[set] ? at[(size_t)set * maxpos + k] : -1; };
    for (int k = 0; k < maxpos; k++)
        for (int set = 0; set < nsets; set++) {
            const int i = launch_at(set, k);
            if (i < 0) continue;
            const hipStream_t st = stream_of(set);
            if (couple == 1 && nsets > 1) {
                for (int t = 0; t < nsets; t++)
                    if (t != set && launch_at(t, k - 1) >= 0) HIPCHK(hipStreamWaitEvent(st, c->lev[launch_at(t, k - 1)], 0));
            } else if (couple == 2 && nsets > 1) {
                if (set > 0 && launch_at(set - 1, k) >= 0) HIPCHK(hipStreamWaitEvent(st, c->lev[launch_at(set - 1, k)], 0));
                if (set + 1 < nsets && launch_at(set + 1, k - 2) >= 0)
                    HIPCHK(hipStreamWaitEvent(st, c->lev[launch_at(set + 1, k - 2)], 0));
            }
            a.slice_base = launches[i].begin;
            a.nslices = launches[i].end - launches[i].begin;
            a.mates = (uint32_t)launches[i].mates;
            if (c->launch_timing) HIPCHK(hipEventRecord(H.l[2 * i], st));
            if (a.nslices) HIPCHK(launch_recon(c->g.cf, launches[i].mcm, a, st));
            {  // the launch's pictures that store their tiles by conversion (TilePlan)
                const auto r = b.post_of[i];
                if (r.second > r.first)
                    HIPCHK(launch_tile_convert(a, c->g.cf, b.d_post + r.first, r.second - r.first, 0, st));
            }
            if (c->launch_timing) HIPCHK(hipEventRecord(H.l[2 * i + 1], st));
            if (couple && nsets > 1) HIPCHK(hipEventRecord(c->lev[i], st));
        }
    for (int set = 0; set < nsets; set++) {
        HIPCHK(hipEventRecord(c->sev[set], stream_of(set)));
        HIPCHK(hipStreamWaitEvent(c->stream, c->sev[set], 0));
    }
    c->last_foot.assign(nsets, std::vector<uint8_t>(c->nslots, 0));
    for (int set = 0; set < nsets && set < (int)b.foot.size(); set++)
        for (int32_t x : b.foot[set]) c->last_foot[set][x] = 1;
    HIPCHK(hipEventRecord(H.b[1], c->stream));
    HIPCHK(hipEventRecord(b.consumed, c->stream));
    b.decoded = true;
    H.nl = c->launch_timing ? nl : 0;
    c->seq++;
    return MP2VG_OK;
}

extern "C" int mp2vg_synchronize(mp2vg_ctx_t* c) {
    if (!c) return MP2VG_E_INVALID;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MP2VG_OK;
}

// time from the earliest set start of batch H to event end
static hipError_t since_earliest_start(const mp2vg_ctx::BatchEv& H, hipEvent_t end, float* ms) {
    float best = 0;
    for (int i = 0; i < H.ns; i++) {
        float t;
        hipError_t e = hipEventElapsedTime(&t, H.s[i], end);
        if (e != hipSuccess) return e;
        best = i == 0 ? t : std::max(best, t);
    }
    *ms = best;
    return hipSuccess;
}

extern "C" int mp2vg_batch_times(mp2vg_ctx_t* c, int32_t back, float* batch_ms, float* launch_ms, int32_t max,
                                 int32_t* count) {
    if (!c || back < 0) return MP2VG_E_INVALID;
    if ((uint64_t)back >= c->seq || back >= mp2vg_ctx::kHist) {
        set_error("no such decoded batch (mp2vg_batch_times keeps the last 64)");
        return MP2VG_E_STATE;
    }
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipStreamSynchronize(c->stream));
    const mp2vg_ctx::BatchEv& H = c->hist[(c->seq - 1 - (uint64_t)back) % mp2vg_ctx::kHist];
    if (batch_ms) HIPCHK(since_earliest_start(H, H.b[1], batch_ms));
    if (count) *count = H.nl;
    for (int i = 0; launch_ms && i < H.nl && i < max; i++)
        HIPCHK(hipEventElapsedTime(&launch_ms[i], H.l[2 * i], H.l[2 * i + 1]));
    return MP2VG_OK;
}

extern "C" int mp2vg_batches_span(mp2vg_ctx_t* c, int32_t back_first, int32_t back_last, float* ms) {
    if (!c || !ms || back_last < 0 || back_first < back_last) return MP2VG_E_INVALID;
    if ((uint64_t)back_first >= c->seq || back_first >= mp2vg_ctx::kHist) {
        set_error("no such decoded batch (mp2vg_batch_times keeps the last 64)");
        return MP2VG_E_STATE;
    }
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipStreamSynchronize(c->stream));
    const mp2vg_ctx::BatchEv& A = c->hist[(c->seq - 1 - (uint64_t)back_first) % mp2vg_ctx::kHist];
    const mp2vg_ctx::BatchEv& B = c->hist[(c->seq - 1 - (uint64_t)back_last) % mp2vg_ctx::kHist];
    HIPCHK(since_earliest_start(A, B.b[1], ms));
    return MP2VG_OK;
}

extern "C" int mp2vg_last_launch_times(mp2vg_ctx_t* c, float* ms, int32_t max, int32_t* count) {
    if (!c) return MP2VG_E_INVALID;
    if (!c->seq) {
        if (count) *count = 0;
        return MP2VG_OK;
    }
    return mp2vg_batch_times(c, 0, nullptr, ms, max, count);
}

extern "C" int mp2vg_last_batch_time(mp2vg_ctx_t* c, float* ms) {
    if (!c || !ms) return MP2VG_E_INVALID;
    if (!c->seq) {
        set_error("no batch decoded");
        return MP2VG_E_STATE;
    }
    return mp2vg_batch_times(c, 0, ms, nullptr, 0, nullptr);
}

extern "C" int mp2vg_download_slot(mp2vg_ctx_t* c, int32_t slot, uint8_t* dst[3], const int32_t dst_stride[3]) {
    if (!c || !dst || slot < 0 || slot >= c->nslots) return MP2VG_E_INVALID;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int p = 0; p < 3; p++) {
        size_t ds = (dst_stride && dst_stride[p]) ? (size_t)dst_stride[p] : (size_t)c->g.pw[p];
        const uint8_t* src = (const uint8_t*)(uintptr_t)c->fptr[slot] + c->g.plane_off[p];
        HIPCHK(hipMemcpy2DAsync(dst[p], ds, src, c->g.stride[p], c->g.pw[p], c->g.ph[p], hipMemcpyDeviceToHost,
                                c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return MP2VG_OK;
}

extern "C" int mp2vg_copy_slot_packed(mp2vg_ctx_t* c, int32_t slot, void* dst, int32_t dst_on_device) {
    if (!c || !dst || slot < 0 || slot >= c->nslots) return MP2VG_E_INVALID;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipStreamSynchronize(c->stream));
    uint8_t* d = (uint8_t*)dst;
    const hipMemcpyKind kind = dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    for (int p = 0; p < 3; p++) {
        const uint8_t* src = (const uint8_t*)(uintptr_t)c->fptr[slot] + c->g.plane_off[p];
        HIPCHK(hipMemcpy2DAsync(d, c->g.pw[p], src, c->g.stride[p], c->g.pw[p], c->g.ph[p], kind, c->stream));
        d += (size_t)c->g.pw[p] * c->g.ph[p];
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return MP2VG_OK;
}

extern "C" int mp2vg_invalidate_slot(mp2vg_ctx_t* c, int32_t slot) {
    if (!c || slot < 0 || slot >= c->nslots) return MP2VG_E_INVALID;
    c->tiles_ok[slot] = 0;  // mp2vg_batch_decode rebuilds them before a batch reads the slot
    return MP2VG_OK;
}

extern "C" int mp2vg_slot_device_ptr(mp2vg_ctx_t* c, int32_t slot, void** dptr) {
    if (!c || !dptr || slot < 0 || slot >= c->nslots) return MP2VG_E_INVALID;
    *dptr = (void*)(uintptr_t)c->fptr[slot];
    return MP2VG_OK;
}

extern "C" int mp2vg_clock_probe(int32_t device, double* ghz) {
    if (!ghz) return MP2VG_E_INVALID;
    HIPCHK(hipSetDevice(device));
    int ncu = 0;
    HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
    unsigned long long* d = nullptr;
    HIPCHK(hipMalloc((void**)&d, 3 * sizeof(unsigned long long)));
    unsigned long long h[3] = {0, 0, 0};
    hipError_t e = hipMemset(d, 0, sizeof(h));
    // 4 waves per SIMD on every CU, ~1 ms of VALU issue
    if (e == hipSuccess) e = launch_clock_probe(d, 1 << 15, ncu * 4, nullptr);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    hipFree(d);
    if (e != hipSuccess || h[1] == 0) return MP2VG_E_HIP;
    *ghz = (double)h[0] / (double)h[1] * 0.1;
    return MP2VG_OK;
}

extern "C" int mp2vg_pool_probe(mp2vg_ctx_t* c, int32_t rw, int32_t reps, double* gbps, int32_t max,
                                int32_t* nblocks) {
    if (!c || !nblocks || max < 0 || (max > 0 && !gbps) || reps <= 0) return MP2VG_E_INVALID;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (hipStream_t s : c->sstreams) HIPCHK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    hipError_t e = hipSuccess;
    if (rw == 5) {  // the record banks: a load sweep over each bank's MB records and coefficient words
        int n = 0;
        for (Bank& bk : c->bank) {
            const std::pair<void*, size_t> bufs[2] = {{bk.d_mbs, bk.cap_mbs * sizeof(mp2vg_mb_t)},
                                                      {bk.d_coefs, bk.cap_coefs * sizeof(uint32_t)}};
            for (const auto& q : bufs) {
                if (n >= max) break;
                float ms = 0;
                if (q.first && q.second >= 16) {
                    e = hipEventRecord(a, c->stream);
                    if (e == hipSuccess) e = launch_block_probe(q.first, q.second & ~(size_t)15, 0, reps, c->d_sink, c->stream);
                    if (e == hipSuccess) e = hipEventRecord(b, c->stream);
                    if (e == hipSuccess) e = hipEventSynchronize(b);
                    if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
                }
                gbps[n++] = ms > 0 ? (double)(q.second & ~(size_t)15) * reps / (ms * 1e6) : 0.0;
                if (e != hipSuccess) break;
            }
        }
        hipEventDestroy(a);
        hipEventDestroy(b);
        if (e != hipSuccess) {
            set_error(std::string("pool probe: ") + hipGetErrorString(e));
            return MP2VG_E_HIP;
        }
        *nblocks = 4;
        return MP2VG_OK;
    }
    if (rw == 2 || rw == 3 || rw == 6 || rw == 7) {  // 2: random 1-KB reads over the pool, 3: many slots at one
                                                      // offset (one rate); 6 / 7: 3 / 2 with each run stored back
        const int waves = 8192, iters = 256;
        float ms = 0;
        if (max > 0 && c->nslots > 0) {
            e = hipEventRecord(a, c->stream);
            for (int r = 0; r < reps && e == hipSuccess; r++)
                e = launch_pool_scatter(c->d_tab, c->nslots, (uint32_t)(c->g.slot_bytes >> 10),
                                        (uint32_t)((2 * c->g.slot_bytes) >> 10),
                                        rw == 3 ? 1 : rw == 6 ? 2 : rw == 7 ? 3 : 0, waves, iters, c->d_sink,
                                        c->stream);
            if (e == hipSuccess) e = hipEventRecord(b, c->stream);
            if (e == hipSuccess) e = hipEventSynchronize(b);
            if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
            gbps[0] = ms > 0 ? (double)waves * iters * 1024 * reps * (rw >= 6 ? 2 : 1) / (ms * 1e6) : 0.0;
        }
        hipEventDestroy(a);
        hipEventDestroy(b);
        if (e != hipSuccess) {
            set_error(std::string("pool probe: ") + hipGetErrorString(e));
            return MP2VG_E_HIP;
        }
        *nblocks = 1;
        return MP2VG_OK;
    }
    const int n = std::min<int>(max, (int)c->chunks.size());
    for (int i = 0; i < n && e == hipSuccess; i++) {
        e = hipEventRecord(a, c->stream);
        if (e == hipSuccess)
            e = rw == 4 ? launch_block_random(c->chunks[i], c->chunk_bytes[i], 8192, 64 * reps, c->d_sink, c->stream)
                        : launch_block_probe(c->chunks[i], c->chunk_bytes[i], rw, reps, c->d_sink, c->stream);
        if (e == hipSuccess) e = hipEventRecord(b, c->stream);
        if (e == hipSuccess) e = hipEventSynchronize(b);
        float ms = 0;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
        const double bytes = rw == 4 ? 8192.0 * 64 * reps * 1024 : (double)(c->chunk_bytes[i] & ~(size_t)15) * reps * (rw ? 2 : 1);
        gbps[i] = ms > 0 ? bytes / (ms * 1e6) : 0.0;
    }
    hipEventDestroy(a);
    hipEventDestroy(b);
    if (e != hipSuccess) {
        set_error(std::string("pool probe: ") + hipGetErrorString(e));
        return MP2VG_E_HIP;
    }
    *nblocks = (int32_t)c->chunks.size();
    return MP2VG_OK;
}

extern "C" int mp2vg_pool_placement(mp2vg_ctx_t* c, float* ms, int32_t max, int32_t* n, int32_t* kept) {
    if (!c || !n || !kept || max < 0 || (max > 0 && !ms)) return MP2VG_E_INVALID;
    *n = (int32_t)c->place_ms.size();
    *kept = c->place_kept;
    for (int i = 0; i < *n && i < max; i++) ms[i] = c->place_ms[i];
    return MP2VG_OK;
}

extern "C" int mp2vg_sink_device_ptr(mp2vg_ctx_t* c, void** dptr) {
    if (!c || !dptr || !c->d_sink) return MP2VG_E_INVALID;
    *dptr = (void*)c->d_sink;
    return MP2VG_OK;
}

extern "C" int mp2vg_slot_digests(mp2vg_ctx_t* c, const int32_t* slots, int32_t n, uint64_t* out) {
    if (!c || !slots || !out || n <= 0) return MP2VG_E_INVALID;
    for (int i = 0; i < n; i++)
        if (slots[i] < 0 || slots[i] >= c->nslots) return MP2VG_E_INVALID;
    HIPCHK(hipSetDevice(c->cfg.device));
    if ((size_t)n > c->cap_digest) {
        hipFree(c->d_dslots);
        hipFree(c->d_digest);
        c->d_dslots = nullptr;
        c->d_digest = nullptr;
        HIPCHK(hipMalloc((void**)&c->d_dslots, sizeof(int32_t) * n));
        HIPCHK(hipMalloc((void**)&c->d_digest, sizeof(unsigned long long) * n));
        c->cap_digest = n;
    }
    HIPCHK(hipMemcpyAsync(c->d_dslots, slots, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(c->d_digest, 0, sizeof(unsigned long long) * n, c->stream));
    int32_t st[3] = {c->g.stride[0], c->g.stride[1], c->g.stride[2]};
    int32_t w[3] = {c->g.pw[0], c->g.pw[1], c->g.pw[2]};
    int32_t h[3] = {c->g.ph[0], c->g.ph[1], c->g.ph[2]};
    HIPCHK(launch_digest(c->d_tab, c->d_dslots, n, c->g.plane_off, st, w, h, c->d_digest, c->stream));
    HIPCHK(hipMemcpyAsync(out, c->d_digest, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MP2VG_OK;
}
