// tiny_mp2v_dec_gpu — the reference CLI sample (tiny_decoder/tiny_mp2v_dec.cpp) written against
// the drop-in header include/mp2v_decoder.h: same decoder_config_t / mp2v_decoder_c / frame_c
// calls, same planar YUV writer and "Time = ... ms" line; the decode runs on the GPU.
//   tiny_mp2v_dec_gpu -v in.m2v -o out.yuv [-w 1920 -h 1088 -c 2 -t 8]
// (the reference sample hard-codes {1920, 1088, 2, 10, 8, true}; those are the defaults here)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mp2v_decoder.h"

static void write_yuv(FILE* fp, frame_c* frame) {
    for (int i = 0; i < 3; i++) {
        uint8_t* plane = frame->get_planes(i);
        for (int y = 0; y < frame->get_height(i); y++, plane += frame->get_strides(i))
            fwrite(plane, 1, frame->get_width(i), fp);
    }
}

int main(int argc, char* argv[]) {
    std::string in, out;
    decoder_config_t cfg = {1920, 1088, 2, 10, 8, true};
    for (int i = 1; i + 1 < argc; i += 2) {
        std::string k = argv[i];
        if (k == "-v") in = argv[i + 1];
        else if (k == "-o") out = argv[i + 1];
        else if (k == "-w") cfg.width = atoi(argv[i + 1]);
        else if (k == "-h") cfg.height = atoi(argv[i + 1]);
        else if (k == "-c") cfg.chroma_format = atoi(argv[i + 1]);
        else if (k == "-t") cfg.num_threads = atoi(argv[i + 1]);
    }
    if (in.empty() || out.empty()) {
        fprintf(stderr, "usage: %s -v in.m2v -o out.yuv [-w W -h H -c chroma_format -t threads]\n", argv[0]);
        return 2;
    }
    FILE* f = fopen(in.c_str(), "rb");
    if (!f) { perror(in.c_str()); return 1; }
    fseek(f, 0, SEEK_END);
    long size = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<uint8_t> buf(((size + 15) & ~15L) + 64, 0);
    if (fread(buf.data(), 1, size, f) != (size_t)size) { perror("read"); return 1; }
    fclose(f);
    FILE* fp = fopen(out.c_str(), "wb");
    if (!fp) { perror(out.c_str()); return 1; }
    mp2v_decoder_c dec(cfg, [fp](frame_c* frame) { write_yuv(fp, frame); });
    const auto start = std::chrono::system_clock::now();
    bool ok = dec.decode(buf.data(), (int)size);
    auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now() - start);
    printf("Time = %.2f ms\n", (double)ms.count());
    fclose(fp);
    if (!ok) fprintf(stderr, "decode failed: %s\n", mp2vg_last_error());
    return ok ? 0 : 1;
}
