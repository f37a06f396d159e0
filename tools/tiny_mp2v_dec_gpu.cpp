// tiny_mp2v_dec_gpu — the reference CLI sample (tiny_decoder/tiny_mp2v_dec.cpp) written against
// the drop-in header include/mp2v_decoder.h: same decoder_config_t / mp2v_decoder_c / frame_c
// calls, same planar YUV writer and "Time = ... ms" line; the decode runs on the GPU.
//   tiny_mp2v_dec_gpu -v in.m2v -o out.yuv [-w 1920 -h 1088 -c 2 -t 8] [-d 0,1,...] [-H headers.json]
// (the reference sample hard-codes {1920, 1088, 2, 10, 8, true}; those are the defaults here)
//   -d  GOP sharding over a device list (mp2vg_decoder_create_multi)
//   -H  after decode(), the decoder's public header members as JSON (the format of
//       oracle/ref_decode's ".hdr.json" mode, which dumps the reference's own members)
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

static void write_headers(FILE* fp, mp2v_decoder_c& dec) {
    const sequence_header_t& sh = dec.m_sequence_header;
    fprintf(fp, "{\"sequence_header\": {\"sequence_header_code\": %u, \"horizontal_size_value\": %u, "
                "\"vertical_size_value\": %u, \"aspect_ratio_information\": %u, \"frame_rate_code\": %u, "
                "\"bit_rate_value\": %u, \"vbv_buffer_size_value\": %u, \"constrained_parameters_flag\": %u, "
                "\"load_intra_quantiser_matrix\": %u, \"load_non_intra_quantiser_matrix\": %u",
            sh.sequence_header_code, sh.horizontal_size_value, sh.vertical_size_value, sh.aspect_ratio_information,
            sh.frame_rate_code, sh.bit_rate_value, sh.vbv_buffer_size_value, sh.constrained_parameters_flag,
            sh.load_intra_quantiser_matrix, sh.load_non_intra_quantiser_matrix);
    const uint8_t* mats[2] = {sh.intra_quantiser_matrix, sh.non_intra_quantiser_matrix};
    const uint32_t loads[2] = {sh.load_intra_quantiser_matrix, sh.load_non_intra_quantiser_matrix};
    const char* names[2] = {"intra_quantiser_matrix", "non_intra_quantiser_matrix"};
    for (int m = 0; m < 2; m++)
        if (loads[m]) {
            fprintf(fp, ", \"%s\": [", names[m]);
            for (int i = 0; i < 64; i++) fprintf(fp, "%s%u", i ? ", " : "", mats[m][i]);
            fprintf(fp, "]");
        }
    const sequence_extension_t& se = dec.m_sequence_extension;
    fprintf(fp, "}, \"sequence_extension\": {\"extension_start_code\": %u, \"extension_start_code_identifier\": %u, "
                "\"profile_and_level_indication\": %u, \"progressive_sequence\": %u, \"chroma_format\": %u, "
                "\"horizontal_size_extension\": %u, \"vertical_size_extension\": %u, \"bit_rate_extension\": %u, "
                "\"vbv_buffer_size_extension\": %u, \"low_delay\": %u, \"frame_rate_extension_n\": %u, "
                "\"frame_rate_extension_d\": %u}, ",
            se.extension_start_code, se.extension_start_code_identifier, se.profile_and_level_indication,
            se.progressive_sequence, se.chroma_format, se.horizontal_size_extension, se.vertical_size_extension,
            se.bit_rate_extension, se.vbv_buffer_size_extension, se.low_delay, se.frame_rate_extension_n,
            se.frame_rate_extension_d);
    if (const sequence_display_extension_t* de = dec.m_sequence_display_extension)
        fprintf(fp, "\"sequence_display_extension\": {\"extension_start_code_identifier\": %u, \"video_format\": %u, "
                    "\"colour_description\": %u, \"colour_primaries\": %u, \"transfer_characteristics\": %u, "
                    "\"matrix_coefficients\": %u, \"display_horizontal_size\": %u, \"display_vertical_size\": %u}, ",
                de->extension_start_code_identifier, de->video_format, de->colour_description, de->colour_primaries,
                de->transfer_characteristics, de->matrix_coefficients, de->display_horizontal_size,
                de->display_vertical_size);
    else
        fprintf(fp, "\"sequence_display_extension\": null, ");
    if (const group_of_pictures_header_t* gh = dec.m_group_of_pictures_header)
        fprintf(fp, "\"group_of_pictures_header\": {\"group_start_code\": %u, \"time_code\": %u, \"closed_gop\": %u, "
                    "\"broken_link\": %u}, ",
                gh->group_start_code, gh->time_code, gh->closed_gop, gh->broken_link);
    else
        fprintf(fp, "\"group_of_pictures_header\": null, ");
    fprintf(fp, "\"sequence_scalable_extension\": %s, \"user_data_len\": %zu}\n",
            dec.m_sequence_scalable_extension ? "1" : "null", dec.user_data.size());
}

int main(int argc, char* argv[]) {
    std::string in, out, hdr_out;
    std::vector<int> devices{0};
    decoder_config_t cfg = {1920, 1088, 2, 10, 8, true};
    for (int i = 1; i + 1 < argc; i += 2) {
        std::string k = argv[i];
        if (k == "-v") in = argv[i + 1];
        else if (k == "-o") out = argv[i + 1];
        else if (k == "-w") cfg.width = atoi(argv[i + 1]);
        else if (k == "-h") cfg.height = atoi(argv[i + 1]);
        else if (k == "-c") cfg.chroma_format = atoi(argv[i + 1]);
        else if (k == "-t") cfg.num_threads = atoi(argv[i + 1]);
        else if (k == "-H") hdr_out = argv[i + 1];
        else if (k == "-d") {
            devices.clear();
            for (const char* p = argv[i + 1]; *p;) {
                devices.push_back(atoi(p));
                while (*p && *p != ',') p++;
                if (*p == ',') p++;
            }
        }
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
    mp2v_decoder_c dec(cfg, [fp](frame_c* frame) { write_yuv(fp, frame); }, devices);
    const auto start = std::chrono::system_clock::now();
    bool ok = dec.decode(buf.data(), (int)size);
    auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now() - start);
    printf("Time = %.2f ms\n", (double)ms.count());
    fclose(fp);
    if (!ok) fprintf(stderr, "decode failed: %s\n", mp2vg_last_error());
    if (ok && !hdr_out.empty()) {
        FILE* hp = fopen(hdr_out.c_str(), "w");
        if (!hp) { perror(hdr_out.c_str()); return 1; }
        write_headers(hp, dec);
        fclose(hp);
    }
    return ok ? 0 : 1;
}
