// mp2v_decoder.h — drop-in C++ declarations of the reference's public decoder API
// (fxslava/tiny_mp2v_dec src/core/decoder.h:25-131), implemented header-only over the C ABI of
// mp2vg.h.  A caller of the reference that only uses
//     decoder_config_t, frame_c::get_planes/get_strides/get_width/get_height,
//     mp2v_decoder_c(const decoder_config_t&, std::function<void(frame_c*)>), decode(buf, len)
// compiles unchanged against this header and links libmp2vg.so instead of the reference library.
//
// Semantics kept from the reference: frames are delivered in display order (B pictures at once,
// I/P delayed by one anchor; decoder.cpp:346-369) on a dedicated render thread; a frame_c is
// valid only while the callback runs; decode() is single-shot and returns after every frame has
// been rendered; the frame layout is the reference frame_c layout (stride = round_up(width, 64)).
// Differences: errors are reported (decode returns false; mp2vg_last_error() has the detail)
// instead of undefined behaviour on out-of-contract input.
#pragma once
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <string>

#include "mp2vg.h"

struct decoder_config_t {
    int width;
    int height;
    int chroma_format;
    int pictures_pool_size;
    int num_threads;
    bool reordering;
};

class frame_c {
public:
    explicit frame_c(const mp2vg_frame_t* f) : m_f(f) {}
    uint8_t* get_planes(int plane_idx) { return m_f->planes[plane_idx]; }
    int get_strides(int plane_idx) { return m_f->stride[plane_idx]; }
    int get_width(int plane_idx) { return m_f->width[plane_idx]; }
    int get_height(int plane_idx) { return m_f->height[plane_idx]; }
    int get_picture_coding_type() const { return m_f->picture_coding_type; }

private:
    const mp2vg_frame_t* m_f;
};

class mp2v_decoder_c {
public:
    mp2v_decoder_c() = default;
    // flags: MP2VG_DECODER_DEVICE_FRAMES hands frames over in HBM (get_planes() then returns
    // device pointers); 0 keeps the reference's host frame_c contract
    mp2v_decoder_c(const decoder_config_t& config, std::function<void(frame_c*)> renderer, int device = 0,
                   int flags = 0) {
        decoder_init(config, renderer, device, flags);
    }
    ~mp2v_decoder_c() {
        if (m_dec) mp2vg_decoder_destroy(m_dec);
    }
    mp2v_decoder_c(const mp2v_decoder_c&) = delete;
    mp2v_decoder_c& operator=(const mp2v_decoder_c&) = delete;

    bool decoder_init(const decoder_config_t& config, std::function<void(frame_c*)> renderer, int device = 0,
                      int flags = 0) {
        m_render = renderer;
        mp2vg_config_t c{};
        c.width = config.width;
        c.height = config.height;
        c.chroma_format = config.chroma_format;
        c.pictures_pool_size = config.pictures_pool_size;
        c.num_threads = config.num_threads;
        c.reordering = config.reordering ? 1 : 0;
        c.device = device;
        c.reserved = flags;
        return mp2vg_decoder_create(&c, &mp2v_decoder_c::trampoline, this, &m_dec) == MP2VG_OK;
    }
    // reference decoder.h:99 — buffer is read as whole ES; returns after all frames rendered
    bool decode(uint8_t* buffer, int len) {
        return m_dec && mp2vg_decoder_decode(m_dec, buffer, (uint64_t)len) == MP2VG_OK;
    }

private:
    static void trampoline(void* user, const mp2vg_frame_t* f) {
        auto* self = static_cast<mp2v_decoder_c*>(user);
        frame_c frame(f);
        if (self->m_render) self->m_render(&frame);
    }
    std::function<void(frame_c*)> m_render;
    mp2vg_decoder_t* m_dec = nullptr;
};
