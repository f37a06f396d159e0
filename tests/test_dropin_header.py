"""CPU: include/mp2v_decoder.h keeps the reference's public C++ surface (decoder.h:25-131) source
compatible: a caller using frame_c(width, height, chroma_format), decoder_init() (twice),
flush(), and the public header members compiles against it unchanged, links libmp2vg.so, and the
parts that need no GPU run: an owned frame_c has the reference frame_c layout
(decoder.cpp:44-77), and without a device decoder_init() fails cleanly instead of crashing."""
import os
import subprocess

from tiny_mp2v_dec_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CALLER = r"""
#include <cassert>
#include <cstdio>
#include <cstdint>
#include "mp2v_decoder.h"

// what a reference caller touches (reference decoder.h:25-131, tiny_mp2v_dec.cpp)
static void reference_style_caller(mp2v_decoder_c& dec, uint8_t* buf, int len) {
    if (dec.decode(buf, len)) {
        const sequence_header_t& sh = dec.m_sequence_header;
        const sequence_extension_t& se = dec.m_sequence_extension;
        sequence_display_extension_t* de = dec.m_sequence_display_extension;
        sequence_scalable_extension_t* ss = dec.m_sequence_scalable_extension;
        group_of_pictures_header_t* gh = dec.m_group_of_pictures_header;
        std::printf("%u %u %u %d %d %d %zu\n", sh.horizontal_size_value, se.chroma_format,
                    gh ? gh->closed_gop : 0u, de != nullptr, ss != nullptr, (int)sh.intra_quantiser_matrix[0],
                    dec.user_data.size());
    }
    dec.flush();
    dec.flush(nullptr);
}

int main() {
    frame_c f(1920, 1088, 1);
    assert(f.get_strides(0) == 1920 && f.get_strides(1) == 960 && f.get_strides(2) == 960);
    assert(f.get_width(1) == 960 && f.get_height(1) == 544 && f.get_height(0) == 1088);
    assert(((uintptr_t)f.get_planes(0) & 31) == 0 && f.get_planes(2) != nullptr);
    f.get_planes(2)[960 * 544 - 1] = 7;  // the whole plane is writable
    frame_c g(176, 144, 2);
    assert(g.get_strides(0) == 192 && g.get_strides(1) == 128 && g.get_height(1) == 144);

    decoder_config_t cfg = {176, 144, 1, 10, 4, true};
    mp2v_decoder_c dec;
    bool a = dec.decoder_init(cfg, [](frame_c*) {});
    bool b = dec.decoder_init(cfg, [](frame_c*) {});  // re-init replaces the decoder
    uint8_t buf[16] = {0};
    reference_style_caller(dec, buf, 16);
    assert(dec.m_sequence_display_extension == nullptr && dec.m_group_of_pictures_header == nullptr);
    std::printf("init %d %d\n", (int)a, (int)b);
    return 0;
}
"""


def test_reference_caller_compiles_links_and_runs(tmp_path):
    src = tmp_path / "caller.cpp"
    src.write_text(CALLER)
    exe = tmp_path / "caller"
    lib_dir = os.path.dirname(_lib.LIB_PATH)
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"), str(src), "-o",
                        str(exe), "-L", lib_dir, "-lmp2vg", f"-Wl,-rpath,{lib_dir}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except ImportError:
        has_gpu = False
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    if not has_gpu:
        assert "init 0 0" in r.stdout
