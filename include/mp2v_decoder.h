// mp2v_decoder.h — drop-in C++ declarations of the reference's public decoder API
// (fxslava/tiny_mp2v_dec src/core/decoder.h:25-131), implemented header-only over the C ABI of
// mp2vg.h.  A caller of the reference that uses
//     decoder_config_t, frame_c(width, height, chroma_format),
//     frame_c::get_planes/get_strides/get_width/get_height,
//     mp2v_decoder_c(const decoder_config_t&, std::function<void(frame_c*)>), decoder_init(...),
//     decode(buf, len), flush(), and the public header members m_sequence_header,
//     m_sequence_extension, m_sequence_display_extension, m_sequence_scalable_extension,
//     m_group_of_pictures_header, user_data
// compiles unchanged against this header and links libmp2vg.so instead of the reference library.
//
// Semantics kept from the reference: frames are delivered in display order (B pictures at once,
// I/P delayed by one anchor; decoder.cpp:346-369) on a dedicated render thread; a frame_c is
// valid only while the callback runs; decode() is single-shot and returns after every frame has
// been rendered; the frame layout is the reference frame_c layout (stride = round_up(width, 64)).
// The header members hold what the reference's decode() leaves in them (mp2v_hdr.cpp:4-83): the
// last sequence header / extension, the last sequence_display_extension and group_of_pictures
// header (nullptr if the stream has none); user_data stays empty, as in the reference, whose
// decode_user_data (decoder.cpp:194-199) stops at the user_data start code it starts on.
// Differences: errors are reported (decode returns false; mp2vg_last_error() has the detail)
// instead of undefined behaviour on out-of-contract input.  Extension: the optional device list
// (GOP sharding over several GPUs, mp2vg_decoder_create_multi).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "mp2vg.h"

struct decoder_config_t {
    int width;
    int height;
    int chroma_format;
    int pictures_pool_size;
    int num_threads;
    bool reordering;
};

// reference mp2v_hdr.h:61-141 type names
using sequence_header_t = mp2vg_sequence_header_t;
using sequence_extension_t = mp2vg_sequence_extension_t;
using sequence_display_extension_t = mp2vg_sequence_display_extension_t;
using sequence_scalable_extension_t = mp2vg_sequence_scalable_extension_t;
using group_of_pictures_header_t = mp2vg_group_of_pictures_header_t;

class frame_c {
public:
    // reference decoder.h:37 / decoder.cpp:44-77: a caller-owned frame in the frame_c layout
    // (planes of height x stride bytes, stride = round_up(width, 64), 32-byte aligned)
    frame_c(int width, int height, int chroma_format) {
        mp2vg_config_t c{};
        c.width = width;
        c.height = height;
        c.chroma_format = chroma_format;
        uint64_t slot = 0;
        if (mp2vg_frame_geometry(&c, m_own.width, m_own.height, m_own.stride, &slot) != MP2VG_OK)
            throw std::invalid_argument("frame_c: unsupported frame geometry");
        for (int i = 0; i < 3; i++) {
            const size_t bytes = (size_t)m_own.height[i] * (size_t)m_own.stride[i];
            m_own.planes[i] = (uint8_t*)std::aligned_alloc(32, (bytes + 31) & ~(size_t)31);
            if (!m_own.planes[i]) throw std::bad_alloc();
        }
        m_f = &m_own;
        m_owned = true;
    }
    explicit frame_c(const mp2vg_frame_t* f) : m_f(f) {}
    ~frame_c() {
        if (m_owned)
            for (auto* p : m_own.planes) std::free(p);
    }
    frame_c(const frame_c&) = delete;
    frame_c& operator=(const frame_c&) = delete;

    uint8_t* get_planes(int plane_idx) { return m_f->planes[plane_idx]; }
    int get_strides(int plane_idx) { return m_f->stride[plane_idx]; }
    int get_width(int plane_idx) { return m_f->width[plane_idx]; }
    int get_height(int plane_idx) { return m_f->height[plane_idx]; }
    int get_picture_coding_type() const { return m_f->picture_coding_type; }
    int get_device() const { return m_f->device; }

private:
    const mp2vg_frame_t* m_f;
    mp2vg_frame_t m_own{};
    bool m_owned = false;
};

class mp2v_picture_c;  // reference decoder.h:57: internal to the decoder, never handed out here

class mp2v_decoder_c {
public:
    mp2v_decoder_c() = default;
    // flags: MP2VG_DECODER_DEVICE_FRAMES hands frames over in HBM (get_planes() then returns
    // device pointers); 0 keeps the reference's host frame_c contract
    mp2v_decoder_c(const decoder_config_t& config, std::function<void(frame_c*)> renderer, int device = 0,
                   int flags = 0) {
        decoder_init(config, renderer, device, flags);
    }
    // GOP sharding over a device list: shard s of the stream -> devices[s % devices.size()]
    mp2v_decoder_c(const decoder_config_t& config, std::function<void(frame_c*)> renderer,
                   const std::vector<int>& devices, int flags = 0) {
        decoder_init(config, renderer, devices, flags);
    }
    ~mp2v_decoder_c() { release(); }
    mp2v_decoder_c(const mp2v_decoder_c&) = delete;
    mp2v_decoder_c& operator=(const mp2v_decoder_c&) = delete;

    bool decoder_init(const decoder_config_t& config, std::function<void(frame_c*)> renderer, int device = 0,
                      int flags = 0) {
        return decoder_init(config, renderer, std::vector<int>{device}, flags);
    }
    bool decoder_init(const decoder_config_t& config, std::function<void(frame_c*)> renderer,
                      const std::vector<int>& devices, int flags = 0) {
        release();  // a second init replaces the decoder (and its GPU context) instead of leaking it
        m_render = renderer;
        mp2vg_config_t c{};
        c.width = config.width;
        c.height = config.height;
        c.chroma_format = config.chroma_format;
        c.pictures_pool_size = config.pictures_pool_size;
        c.num_threads = config.num_threads;
        c.reordering = config.reordering ? 1 : 0;
        c.device = devices.empty() ? 0 : devices[0];
        c.reserved = flags;
        std::vector<int32_t> dev(devices.begin(), devices.end());
        if (dev.empty()) dev.push_back(0);
        return mp2vg_decoder_create_multi(&c, dev.data(), (int32_t)dev.size(), &mp2v_decoder_c::trampoline, this,
                                          &m_dec) == MP2VG_OK;
    }
    // reference decoder.h:99 — buffer is read as whole ES; returns after all frames rendered
    bool decode(uint8_t* buffer, int len) {
        if (!m_dec || mp2vg_decoder_decode(m_dec, buffer, (uint64_t)(len < 0 ? 0 : len)) != MP2VG_OK) return false;
        mp2vg_stream_headers_t h{};
        mp2vg_decoder_stream_headers(m_dec, &h);
        m_sequence_header = h.sequence_header;
        m_sequence_extension = h.sequence_extension;
        m_display = h.sequence_display_extension;
        m_gop = h.group_of_pictures_header;
        m_sequence_display_extension = h.have_sequence_display_extension ? &m_display : nullptr;
        m_group_of_pictures_header = h.have_group_of_pictures_header ? &m_gop : nullptr;
        return true;
    }
    // reference decoder.h:100: submits the last picture and drains the output.  decode() already
    // does both before it returns, so there is never anything left to flush.
    void flush(mp2v_picture_c* cur_pic = nullptr) { (void)cur_pic; }

    // headers & user data (reference decoder.h:124-130)
    std::vector<uint8_t> user_data;
    sequence_header_t m_sequence_header = {};
    sequence_extension_t m_sequence_extension = {};
    sequence_display_extension_t* m_sequence_display_extension = nullptr;
    sequence_scalable_extension_t* m_sequence_scalable_extension = nullptr;  // scalable streams are rejected
    group_of_pictures_header_t* m_group_of_pictures_header = nullptr;

private:
    void release() {
        if (m_dec) mp2vg_decoder_destroy(m_dec);
        m_dec = nullptr;
    }
    static void trampoline(void* user, const mp2vg_frame_t* f) {
        auto* self = static_cast<mp2v_decoder_c*>(user);
        frame_c frame(f);
        if (self->m_render) self->m_render(&frame);
    }
    std::function<void(frame_c*)> m_render;
    mp2vg_decoder_t* m_dec = nullptr;
    sequence_display_extension_t m_display = {};
    group_of_pictures_header_t m_gop = {};
};
