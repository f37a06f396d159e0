/*
 * mp2vg.h — C ABI of the MI355X-native MPEG-2 macroblock reconstruct path.
 *
 * Plain C, plain pointers and sizes, int status codes; no torch / HIP types in any signature.
 * The shared library is tiny_mp2v_dec_amd/_build/libmp2vg.so (hipcc, gfx950).
 *
 * What each group of entry points replaces in the reference (fxslava/tiny_mp2v_dec):
 *
 *   mp2vg_create / mp2vg_destroy / mp2vg_frame_geometry
 *       replace decoder_init's frame pool (reference src/core/decoder.cpp:381-406) and the
 *       frame_c plane layout (decoder.h:34-49, decoder.cpp:44-77): 3 planes per picture,
 *       stride = round_up(width, 64), chroma stride = round_up(stride/2, 64) (4:4:4: = stride).
 *   mp2vg_batch_upload / mp2vg_batch_decode
 *       replace the per-slice hot loop `do { m_parse_macroblock_func(&bs, cache); } while(...)`
 *       (decoder.cpp:148-150) — i.e. everything parse_macroblock_template does AFTER parsing:
 *       MC (mb_decoder.cpp:291-339 -> mc.cpp tables -> mc_sse2.hpp), dequant + mismatch control
 *       (parse_block, mb_decoder.cpp:74-155), SSE2 IDCT put/add (idct_sse2.hpp:96-120) and
 *       block placement (mb_decoder.cpp:166-196) — for a whole batch of pictures per call.
 *       The seam is the packed record stream defined below (SURVEY.md §8b "Record stream").
 *   mp2vg_parse_es
 *       the host record emitter: start-code scan + header parse + VLC/MV/DC parse
 *       (decoder.cpp:278-329, mp2v_hdr.cpp, mp2v_vlc_dec.hpp, mb_decoder.cpp:341-641) producing
 *       records instead of pixels.
 *   mp2vg_decoder_*
 *       the drop-in decoder: mp2v_decoder_c(config, renderer) + decode(buf, len) with frames
 *       delivered in display order on a render thread (decoder.h:82-131, decoder.cpp:346-379).
 *       include/mp2v_decoder.h wraps these in the reference's own C++ class names.
 */
#ifndef MP2VG_H
#define MP2VG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: coefficient words carry the MB column mod 8 in bits 26-28 and the FIRST1S / DC flags in
 *    bits 29 / 30 (1: FIRST1S bit 26, DC bit 27, MB column bits 28-30); mp2vg_frame_t.device */
#define MP2VG_ABI_VERSION 2

/* ---- status codes --------------------------------------------------------------------- */
enum {
    MP2VG_OK = 0,
    MP2VG_E_INVALID = -1,     /* bad argument / malformed record batch                    */
    MP2VG_E_UNSUPPORTED = -2, /* stream outside the reference's decodable subset */
    MP2VG_E_HIP = -3,         /* HIP runtime error (no device, launch failure, ...)        */
    MP2VG_E_NOMEM = -4,
    MP2VG_E_STATE = -5,       /* call out of order                                           */
    MP2VG_E_BITSTREAM = -6    /* bitstream syntax error                                      */
};

/* ---- record stream (the seam; 32-byte MB records + 4-byte coefficient words) -------------
 *
 * One record per macroblock of every picture, skipped MBs included (as MC-only records), in
 * raster order: picture p owns records [mb_first, mb_first + mb_width*mb_height).
 * Motion vectors are FINAL luma vectors after all PMV rules and skipped-MB quirks
 * (reference mb_decoder.cpp:447-519, 541-550, 580-604); chroma scaling stays on the device
 * (mb_decoder.cpp:198-206).
 */
enum {
    MP2VG_MB_INTRA = 1u << 0,     /* IDCT put, no MC; cbp codes every block, and every MB of an
                                     I picture is intra (both checked on upload)               */
    MP2VG_MB_FWD = 1u << 1,       /* forward prediction from fwd_slot                        */
    MP2VG_MB_BWD = 1u << 2,       /* backward prediction from bwd_slot (both bits: bidir avg) */
    MP2VG_MB_FIELD_MC = 1u << 3,  /* frame picture, field prediction: 2 vectors, 16x8 each  */
    MP2VG_MB_DCT_FIELD = 1u << 4  /* dct_type = 1 (field DCT block placement)               */
};
/* motion_vertical_field_select[r][s] lives in flags bit (8 + 2*r + s) */
#define MP2VG_MB_FS_BIT(r, s) (1u << (8 + 2 * (r) + (s)))

typedef struct mp2vg_mb {
    uint16_t x, y;        /* macroblock column / row                                          */
    uint16_t flags;       /* MP2VG_MB_* | field selects                                        */
    uint16_t cbp;         /* coded block pattern, bit b <-> block b (mb_decoder.cpp:421-445)   */
    uint8_t  qscale;      /* quantiser_scale after q_scale_type mapping (decoder.cpp:140-145)  */
    uint8_t  reserved;
    uint16_t ncoef;       /* number of coefficient words                                        */
    uint32_t coef_off;    /* index of the first coefficient word in the batch's coef array     */
    int16_t  mv[2][2][2]; /* [vector r][direction s: 0 fwd, 1 bwd][x, y], half-pel luma units;
                             field-MC vertical components in field units                       */
} mp2vg_mb_t;             /* 32 bytes */

/* Coefficient word: bits 0-15 int16 level (signed run-level level, or the final QFS[0] value
 * when MP2VG_COEF_DC), bits 16-21 scan position i (0..63), bits 22-25 block index (0..11),
 * bits 26-28: the MB's column x mod 8 (bits 22-27 are the word's (MB in its 4-MB group, block)
 * index for the kernel; mp2vg_batch_upload validates them), bit 29 FIRST1S: non-intra first
 * coefficient coded with the B.14 '1s' code — dequantised as (3*W[0]*qs)>>5 without the
 * +-2047 clamp (mb_decoder.cpp:79-88), bit 30 DC: intra DC value, excluded from the mismatch
 * parity (mb_decoder.cpp:76,160), bit 31: 0.  FIRST1S and DC words carry i = 0.
 * Words of one MB are grouped by block, blocks in bitstream order.                           */
#define MP2VG_COEF_LEVEL(w) ((int16_t)((w) & 0xffffu))
#define MP2VG_COEF_POS(w) (((w) >> 16) & 63u)
#define MP2VG_COEF_BLOCK(w) (((w) >> 22) & 15u)
#define MP2VG_COEF_FIRST1S (1u << 29)
#define MP2VG_COEF_DC (1u << 30)
#define MP2VG_COEF_MBX(x) (((uint32_t)(x) & 7u) << 26)
#define MP2VG_COEF_PACK(level, pos, block, fl) \
    ((uint32_t)(uint16_t)(int16_t)(level) | ((uint32_t)(pos) << 16) | ((uint32_t)(block) << 22) | (uint32_t)(fl))

typedef struct mp2vg_picture {
    int32_t  dst_slot;            /* frame-pool slot written                                   */
    int32_t  fwd_slot;            /* forward reference slot (L0), -1 = none                    */
    int32_t  bwd_slot;            /* backward reference slot (L1), -1 = none                   */
    int32_t  picture_coding_type; /* 1 I, 2 P, 3 B                                              */
    uint32_t mb_first;            /* first MB record of this picture                            */
    uint16_t mb_width, mb_height;
    uint8_t  alternate_scan;
    uint8_t  reserved0[3];
    int32_t  temporal_reference;
    uint8_t  W[4][64];            /* quantiser matrices in scan order: [0] intra, [1] non-intra,
                                     [2] chroma intra, [3] chroma non-intra (decoder.cpp:154-192) */
} mp2vg_picture_t;                /* 288 bytes */

/* ---- device context ------------------------------------------------------------------- */
typedef struct mp2vg_config {
    int32_t width, height;       /* CODED size (multiples of 16), as the reference's config  */
    int32_t chroma_format;       /* 1 = 4:2:0, 2 = 4:2:2, 3 = 4:4:4                          */
    int32_t pictures_pool_size;  /* number of device frame slots                             */
    int32_t num_threads;         /* host parse threads (0 = auto)                            */
    int32_t reordering;          /* display reorder in the drop-in decoder                   */
    int32_t device;              /* HIP device ordinal                                       */
    int32_t reserved;            /* flags: MP2VG_DECODER_* (drop-in decoder), MP2VG_CTX_*     */
} mp2vg_config_t;

/* mp2vg_config_t.reserved flag for mp2vg_decoder_create: frames are handed to the renderer in
 * HBM (mp2vg_frame_t.planes are device pointers on cfg->device, valid during the callback), with
 * no PCIe download: the opt-in device-pointer output path for callers that consume frames on the
 * GPU.  Without it, planes are host memory (the reference's frame_c contract). */
#define MP2VG_DECODER_DEVICE_FRAMES 1
/* mp2vg_config_t.reserved flag for mp2vg_create: run every picture set of a batch on one stream
 * (default: closed groups of pictures dealt to 2 streams, or MP2VG_STREAMS), so per-launch
 * device times never overlap -- per-kernel roofline measurements and their rocprof traces */
#define MP2VG_CTX_ONE_STREAM 2

typedef struct mp2vg_ctx mp2vg_ctx_t;

int  mp2vg_abi_version(void);
const char* mp2vg_status_string(int status);
const char* mp2vg_last_error(void); /* thread-local detail of the last failure */

int  mp2vg_create(const mp2vg_config_t* cfg, mp2vg_ctx_t** out);
int  mp2vg_destroy(mp2vg_ctx_t* ctx);
/* plane geometry of every frame slot: width/height/stride of plane 0..2, bytes per slot */
int  mp2vg_frame_geometry(const mp2vg_config_t* cfg, int32_t width[3], int32_t height[3],
                          int32_t stride[3], uint64_t* slot_bytes);
/* grow the frame pool to nslots slots (new slots read as zero).  Slots live in blocks of 16, each
 * its own allocation, with each slot's anchor tiles (the motion-compensation taps' copy of I and
 * P pictures, 2 x slot bytes); slot addresses are not contiguous: mp2vg_slot_device_ptr */
int  mp2vg_reserve_slots(mp2vg_ctx_t* ctx, int32_t nslots);

/* Upload a record batch from host memory (staged through pinned buffers, hipMemcpyAsync on the
 * context stream).  The batch stays resident in HBM until the next upload. */
int  mp2vg_batch_upload(mp2vg_ctx_t* ctx, const mp2vg_picture_t* pics, int32_t npics,
                        const mp2vg_mb_t* mbs, uint64_t nmbs, const uint32_t* coefs,
                        uint64_t ncoefs);
/* Host-only check of a record batch against a geometry and a pool of nslots slots: exactly the
 * validation and planning mp2vg_batch_upload runs before any copy (no device needed).  Returns
 * MP2VG_OK, or MP2VG_E_INVALID with the reason in mp2vg_last_error().  Optional outputs (NULL to
 * skip): *nlaunches = kernel launches per mp2vg_batch_decode; launch_of_pic[npics] = the launch
 * (index into mp2vg_batch_times' launch list) that reconstructs each picture; launch_mode[i <
 * max_launches] = that launch's kernel (0 I, 1 P, 2 B, 3 mixed P/B picture types, 4 I without tile stores). */
int  mp2vg_batch_validate(const mp2vg_config_t* cfg, int32_t nslots, const mp2vg_picture_t* pics,
                          int32_t npics, const mp2vg_mb_t* mbs, uint64_t nmbs,
                          const uint32_t* coefs, uint64_t ncoefs, int32_t* nlaunches,
                          int32_t* launch_of_pic, int32_t* launch_mode, int32_t max_launches);
/* Enqueue the reconstruct of every picture of the resident batch: pictures are grouped by
 * reference-dependency depth and each depth level is one kernel launch (one workgroup per
 * slice = MB row).  Asynchronous; per-launch device times are recorded with HIP events. */
int  mp2vg_batch_decode(mp2vg_ctx_t* ctx);
int  mp2vg_synchronize(mp2vg_ctx_t* ctx);
/* number of kernel launches of the last mp2vg_batch_decode and their device times (ms) */
int  mp2vg_last_launch_times(mp2vg_ctx_t* ctx, float* ms, int32_t max, int32_t* count);
/* device time (ms) of the whole last mp2vg_batch_decode: first launch start to last launch end */
int  mp2vg_last_batch_time(mp2vg_ctx_t* ctx, float* ms);
/* times of the batch decoded `back` decodes ago (0 = the last; the last 64 are kept), so batches
 * can be decoded back to back and timed afterwards: whole-batch span (batch_ms, may be NULL) and
 * per-launch device times (launch_ms[0..min(count, max)), may be NULL); synchronises */
int  mp2vg_batch_times(mp2vg_ctx_t* ctx, int32_t back, float* batch_ms, float* launch_ms, int32_t max,
                       int32_t* count);
/* device time (ms) from the start of the batch decoded `back_first` decodes ago to the end of the
 * one `back_last` decodes ago (back_first >= back_last; the last 64 are kept): the device span of
 * back-to-back batches, whose picture sets overlap across batch boundaries; synchronises */
int  mp2vg_batches_span(mp2vg_ctx_t* ctx, int32_t back_first, int32_t back_last, float* ms);
/* copy one frame slot to host planes (each plane written width x height, tightly packed if
 * dst_stride is 0); synchronous */
int  mp2vg_download_slot(mp2vg_ctx_t* ctx, int32_t slot, uint8_t* dst_planes[3],
                         const int32_t dst_stride[3]);
/* copy one frame slot's visible planes Y, U, V tightly packed (the reference sample's write_yuv
 * layout, tiny_mp2v_dec.cpp:11-17) to dst: HBM of the context's device when dst_on_device
 * (e.g. an RCCL send buffer for the rank-0 frame gather), else host memory; synchronous */
int  mp2vg_copy_slot_packed(mp2vg_ctx_t* ctx, int32_t slot, void* dst, int32_t dst_on_device);
/* raw device pointer of a slot (for in-HBM consumers such as a digest kernel or RCCL).  The
 * slot is READ-ONLY for callers: the motion-compensation taps read a reference from its anchor
 * tiles, a second copy the decode writes next to the frame (recon.hip), so bytes written through
 * this pointer are not seen by later predictions unless the caller then calls
 * mp2vg_invalidate_slot, which makes the next decode that reads the slot rebuild its tiles.
 * The pointer can change once, at the context's first mp2vg_batch_decode, when the pool's
 * placement calibration keeps a copy of the pool (mp2vg_pool_placement; contents are carried
 * over): fetch it after that decode, or turn the calibration off (MP2VG_PLACE_CANDIDATES=1). */
int  mp2vg_slot_device_ptr(mp2vg_ctx_t* ctx, int32_t slot, void** dptr);
/* the slot's frame was written by someone other than the decode (an RCCL receive, an external
 * producer writing through mp2vg_slot_device_ptr): its anchor tiles are stale.  The next batch
 * that predicts from the slot rebuilds them from the frame first (tile_convert).  Call it after
 * the writes have completed and before mp2vg_batch_decode of a batch that reads the slot. */
int  mp2vg_invalidate_slot(mp2vg_ctx_t* ctx, int32_t slot);
/* The pool's placement calibration (runtime.cpp calibrate_placement): at the first batch of a
 * context whose pool holds at least MP2VG_PLACE_MIN_MB (4096) MB, the batch is
 * decoded on the pool and on MP2VG_PLACE_CANDIDATES - 1 (default 2) copies of it in freshly
 * allocated blocks, and the pool with the shortest batch is kept; every candidate ends in the
 * same state, so no output changes.  The other candidates stay allocated until mp2vg_destroy
 * while an eighth of the device memory stays free (freeing them slowed the kept pool;
 * MP2VG_PLACE_HOLD=0 frees them).  MP2VG_PLACE_CANDIDATES=1 turns it off.  This returns the
 * measured batch times (ms[0..n): round 0 of each candidate, then round 1; n = 0 when it did not
 * run) and the candidate kept (0 = the pool as first allocated, -1 = none). */
int  mp2vg_pool_placement(mp2vg_ctx_t* ctx, float* ms, int32_t max, int32_t* n, int32_t* kept);
/* diagnostics: device address of the context's kernel sink block (dummy loads and stores of the
 * decode; from +3072 the per-stage cycle sums of a stamp build, tools/stamps.py).  Never written
 * by callers. */
int  mp2vg_sink_device_ptr(mp2vg_ctx_t* ctx, void** dptr);
/* diagnostics: the device's shader clock (GHz) while every SIMD issues VALU for ~1 ms (s_memtime
 * against the 100-MHz s_memrealtime); bench.py records it per box.  Synchronises the device. */
int  mp2vg_clock_probe(int32_t device, double* ghz);
/* the host threads a decoder uses when num_threads = 0: the hardware threads, capped by the
 * process's affinity mask and a cgroup v2 CPU quota (cpu.max); no device needed */
int  mp2vg_cpu_budget(void);
/* diagnostics (pool placement, tools/placement.py): per pool block (frames and tiles of 16 slots
 * each, in allocation order: frames, tiles, frames, ...) the HBM rate in GB/s of `reps` sweeps
 * that load every 16-B word and, with rw = 1, store it back unchanged.  gbps[i] for the first
 * `max` blocks; *nblocks = the pool's block count.  rw = 2: one rate (gbps[0], *nblocks = 1) for
 * 1-KB reads at random slots and offsets over the whole pool; rw = 3: the same with many slots read
 * at one offset at a time; rw = 4: per block, random 1-KB reads inside the block; rw = 5: load
 * sweeps over the two record banks (MB records, coefficient words: 4 rates, 0 where a bank is
 * not allocated); rw = 6 / 7: rw = 3 / 2 with each 1-KB run stored back unchanged.  Synchronises
 * the context; contents kept. */
int  mp2vg_pool_probe(mp2vg_ctx_t* ctx, int32_t rw, int32_t reps, double* gbps, int32_t max, int32_t* nblocks);
/* 64-bit order-independent digest of each listed slot's visible planes, computed on device:
 * sum over visible dwords d at (row, byte_x) of mix64(mix64((row << 32) | byte_x) ^ d) mod 2^64
 * (numpy twin: tiny_mp2v_dec_amd.records.planes_digest) */
int  mp2vg_slot_digests(mp2vg_ctx_t* ctx, const int32_t* slots, int32_t n, uint64_t* out);

/* ---- stream headers ----------------------------------------------------------------------
 * The sequence-level headers the reference keeps as public members of mp2v_decoder_c
 * (decoder.h:124-130), with the reference's field names (mp2v_hdr.h:61-141) and parsed the way
 * the reference parses them (mp2v_hdr.cpp:4-83): a later header of the same kind overwrites an
 * earlier one, the matrices are the 64 bytes as transmitted, fields a header does not carry stay
 * 0, and the start-code fields hold the 32-bit start code (extension_start_code stays 0, as the
 * reference never sets it).  Scalable extensions are outside the decodable subset (rejected). */
typedef struct mp2vg_sequence_header {
    uint32_t sequence_header_code, horizontal_size_value, vertical_size_value, aspect_ratio_information,
             frame_rate_code, bit_rate_value, vbv_buffer_size_value, constrained_parameters_flag,
             load_intra_quantiser_matrix;
    uint8_t  intra_quantiser_matrix[64];
    uint32_t load_non_intra_quantiser_matrix;
    uint8_t  non_intra_quantiser_matrix[64];
} mp2vg_sequence_header_t;
typedef struct mp2vg_sequence_extension {
    uint32_t extension_start_code, extension_start_code_identifier, profile_and_level_indication,
             progressive_sequence, chroma_format, horizontal_size_extension, vertical_size_extension,
             bit_rate_extension, vbv_buffer_size_extension, low_delay, frame_rate_extension_n,
             frame_rate_extension_d;
} mp2vg_sequence_extension_t;
typedef struct mp2vg_sequence_display_extension {
    uint32_t extension_start_code_identifier, video_format, colour_description, colour_primaries,
             transfer_characteristics, matrix_coefficients, display_horizontal_size, display_vertical_size;
} mp2vg_sequence_display_extension_t;
typedef struct mp2vg_sequence_scalable_extension {
    uint32_t extension_start_code_identifier, scalable_mode, layer_id, lower_layer_prediction_horizontal_size,
             lower_layer_prediction_vertical_size, horizontal_subsampling_factor_m,
             horizontal_subsampling_factor_n, vertical_subsampling_factor_m, vertical_subsampling_factor_n,
             picture_mux_enable, mux_to_progressive_sequence, picture_mux_order, picture_mux_factor;
} mp2vg_sequence_scalable_extension_t;
typedef struct mp2vg_group_of_pictures_header {
    uint32_t group_start_code, time_code, closed_gop, broken_link;
} mp2vg_group_of_pictures_header_t;
typedef struct mp2vg_stream_headers {
    int32_t have_sequence_display_extension;  /* reference: m_sequence_display_extension != nullptr */
    int32_t have_group_of_pictures_header;    /* reference: m_group_of_pictures_header != nullptr   */
    mp2vg_sequence_header_t sequence_header;
    mp2vg_sequence_extension_t sequence_extension;
    mp2vg_sequence_display_extension_t sequence_display_extension;
    mp2vg_group_of_pictures_header_t group_of_pictures_header; /* the last one in the stream      */
} mp2vg_stream_headers_t;

/* ---- host record emitter -------------------------------------------------------------- */
typedef struct mp2vg_parsed mp2vg_parsed_t;

/* Parse a whole elementary stream into records.  Pictures are numbered in decode order and
 * slot ids are decode indices (dst_slot = i; refs point at earlier indices).  Validates the
 * reference's input contract and returns MP2VG_E_UNSUPPORTED outside it. */
int  mp2vg_parse_es(const uint8_t* buf, uint64_t len, const mp2vg_config_t* cfg,
                    mp2vg_parsed_t** out);
int  mp2vg_parsed_counts(const mp2vg_parsed_t* p, int32_t* npics, uint64_t* nmbs,
                         uint64_t* ncoefs);
const mp2vg_picture_t* mp2vg_parsed_pictures(const mp2vg_parsed_t* p);
const mp2vg_mb_t*      mp2vg_parsed_mbs(const mp2vg_parsed_t* p);
const uint32_t*        mp2vg_parsed_coefs(const mp2vg_parsed_t* p);
/* display order (decode indices), as the reference's output scheduler emits them */
int  mp2vg_parsed_display_order(const mp2vg_parsed_t* p, int32_t* order, int32_t n);
/* GOP index (0-based, by group_start_code) of each picture, for GOP sharding */
int  mp2vg_parsed_gop_index(const mp2vg_parsed_t* p, int32_t* gop, int32_t n);
/* sequence headers of the parsed stream (see mp2vg_stream_headers_t) */
int  mp2vg_parsed_stream_headers(const mp2vg_parsed_t* p, mp2vg_stream_headers_t* out);
/* Independent shards for GOP sharding: shard[i] of each picture (decode order), numbered from 0.
 * A shard is a maximal run of pictures, in decode order, that no later picture predicts across:
 * a closed GOP (or several open GOPs chained by their leading B pictures), since a picture's
 * references are only the two latest anchors (reference decoder.cpp:299-304).  The B pictures
 * between the first two anchors of a GOP whose header has closed_gop = 1 predict backward only
 * (ISO/IEC 13818-2 6.3.8), so their picture-level forward anchor (the previous GOP's last one,
 * reference decoder.cpp:299-304) does not join the shards; the multi-device decoder refuses
 * (MP2VG_E_UNSUPPORTED) such a picture if a macroblock of it does predict forward.  Returns the
 * number of shards. */
int  mp2vg_parsed_shards(const mp2vg_parsed_t* p, int32_t* shard, int32_t n);
void mp2vg_parsed_free(mp2vg_parsed_t* p);

/* Conformance hook: decode one Annex B code (MSB-first 64-bit window: the code, then whatever
 * follows) with the emitter's own decoders.  Tables follow the reference's VLC decoders
 * (mp2v_vlc_dec.hpp:36-267) except where the emitter reads more: MOTION consumes the sign bit
 * and returns the signed motion_code; COEF_B14/B15 consume the sign bit (or the escape's run
 * and level) and return run in *value and the signed level in *aux (EOB: *value = -1); MBA
 * returns -33 for macroblock_escape.  Returns MP2VG_E_BITSTREAM for an invalid code. */
enum {
    MP2VG_VLC_MBA = 0, MP2VG_VLC_MBTYPE_I = 1, MP2VG_VLC_MBTYPE_P = 2, MP2VG_VLC_MBTYPE_B = 3,
    MP2VG_VLC_CBP = 4, MP2VG_VLC_MOTION = 5, MP2VG_VLC_DC_LUMA = 6, MP2VG_VLC_DC_CHROMA = 7,
    MP2VG_VLC_COEF_B14 = 8, MP2VG_VLC_COEF_B15 = 9
};
int  mp2vg_vlc_decode(int32_t table, uint64_t bits, int32_t* value, int32_t* aux, int32_t* consumed);

/* ---- synthetic stream writer (the accepted subset only) --------------------- */
typedef struct mp2vg_gen_params {
    int32_t width, height, chroma_format;
    int32_t n_gops;              /* closed GOPs                                              */
    int32_t gop_n, gop_m;        /* N (pictures per GOP), M (anchor distance); M=1 -> no B  */
    uint32_t seed;
    int32_t frame_pred_frame_dct;/* 1: frame MC/DCT only; 0: field MC + field DCT allowed   */
    int32_t alternate_scan;      /* 0, 1, or -1 = random per picture                        */
    int32_t q_scale_type;        /* 0, 1, or -1 = random per picture                        */
    int32_t intra_dc_precision;  /* 0..3, or -1 = random per picture                        */
    int32_t coefs_min, coefs_max;/* AC coefficients per coded block                         */
    int32_t intra_coefs_min, intra_coefs_max;
    int32_t big_level_permille;  /* probability (per 1000) of a large escape level          */
    int32_t escape_permille;     /* probability of forcing an escape code                   */
    int32_t quant_permille;      /* probability an MB carries a new quantiser_scale         */
    int32_t f_code;              /* motion f_code (1..9)                                     */
    int32_t mix;                 /* 0: SURVEY §8d C2 mix; 1: intra only; 2: MC-heavy         */
    int32_t leading_b;           /* closed GOP starts I + (M-1) backward-only B pictures    */
    int32_t big_matrix_permille; /* probability of a quantiser-matrix entry > 128           */
    int32_t reserved[5];
} mp2vg_gen_params_t;

void mp2vg_gen_default_params(mp2vg_gen_params_t* p);
int  mp2vg_generate_es(const mp2vg_gen_params_t* p, uint8_t** out, uint64_t* len);
void mp2vg_free(void* ptr);

/* ---- drop-in decoder (reference mp2v_decoder_c) ---------------------------------------- */
typedef struct mp2vg_frame {
    uint8_t* planes[3];       /* host copy (device pointer with MP2VG_DECODER_DEVICE_FRAMES),
                                 valid only during the callback (frame_c rule)               */
    int32_t  width[3], height[3], stride[3];
    int32_t  picture_coding_type;
    int32_t  decode_index;
    int32_t  device;          /* HIP device that decoded the frame (its planes' device with
                                 MP2VG_DECODER_DEVICE_FRAMES)                                 */
} mp2vg_frame_t;
typedef void (*mp2vg_render_fn)(void* user, const mp2vg_frame_t* frame);
typedef struct mp2vg_decoder mp2vg_decoder_t;

int  mp2vg_decoder_create(const mp2vg_config_t* cfg, mp2vg_render_fn fn, void* user,
                          mp2vg_decoder_t** out);
/* The drop-in decoder over several devices (GOP sharding): the independent shards of a stream
 * (mp2vg_parsed_shards) are merged in decode order into runs of at least one decode chunk (16
 * pictures: consecutive shards join a run until it is that long) and the runs are dealt
 * round-robin, run r -> devices[r % ndevices], each device
 * decoding its shards with its own frame pool, record banks and streams, concurrently; frames
 * reach the renderer in the stream's display order whatever device decoded them.  cfg->device is
 * ignored; a device may be listed more than once (e.g. {0, 0}: two independent lanes on one GPU).
 * The reference's picture-parallel runtime this replaces: threads.cpp:22-36, 120-186 and
 * decoder.cpp:299-304, 346-379.  ndevices = 1 is mp2vg_decoder_create on devices[0]. */
int  mp2vg_decoder_create_multi(const mp2vg_config_t* cfg, const int32_t* devices, int32_t ndevices,
                                mp2vg_render_fn fn, void* user, mp2vg_decoder_t** out);
/* decode a whole elementary stream (reference decode(): single-shot, synchronous; frames are
 * delivered in display order to fn on a dedicated render thread before this returns) */
int  mp2vg_decoder_decode(mp2vg_decoder_t* dec, const uint8_t* buf, uint64_t len);
/* sequence headers of the last decoded stream (reference public members, decoder.h:124-130) */
int  mp2vg_decoder_stream_headers(const mp2vg_decoder_t* dec, mp2vg_stream_headers_t* out);
/* frames decoded by each lane of the decoder in its last decode() (lane i = devices[i]); returns
 * the number of lanes */
int  mp2vg_decoder_lane_frames(const mp2vg_decoder_t* dec, int32_t* frames, int32_t n);
/* frame buffers the decoder's frame pools hold (host + device): 2 * 16 + 4 per lane unless a
 * renderer that holds no frame had to wait for display order (then the pool grows) */
int  mp2vg_decoder_frames_allocated(const mp2vg_decoder_t* dec);
/* lane hand-offs in the last decode() (several lanes): in_flight = times the stream moved to
 * another lane while the lane just left was still downloading its last chunk (the host did not
 * wait: both lanes' chunks in flight at once); blocks = times the host waited for another lane's
 * downloads because the frame pool could not give the next chunk its frames otherwise; landed =
 * lane changes where the lane just left had nothing in flight or its downloads were found landed
 * by the non-blocking check; changes = lane changes.  Every change is in_flight, landed or one of
 * the blocks.  Any out pointer may be NULL. */
int  mp2vg_decoder_handoff_stats(const mp2vg_decoder_t* dec, int32_t* in_flight, int32_t* blocks, int32_t* landed,
                                 int32_t* changes);
int  mp2vg_decoder_destroy(mp2vg_decoder_t* dec);

#ifdef __cplusplus
}
#endif
#endif /* MP2VG_H */
