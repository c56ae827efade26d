/*
 * omr_oracle.h — CPU restatement of the reference's rendering path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline — never as the product path.  See omr_oracle.c for the semantics table.
 */
#ifndef OMR_ORACLE_H
#define OMR_ORACLE_H

#include "omr/omr.h"

#ifdef __cplusplus
extern "C" {
#endif

int64_t oracle_java_round(double a);
int32_t oracle_quantize(double x, const omr_channel_binding* cb, const omr_quantum_def* q);
omr_status oracle_build_lut(const omr_channel_binding* cb, const omr_quantum_def* q,
                            uint8_t* lut, int64_t n);
omr_status oracle_render_packed_int(const omr_quantum_def* q, const omr_channel_binding* ch,
                                    int32_t size_c, const void* const* planes,
                                    int64_t row_stride, int32_t pixel_type, int32_t big_endian,
                                    int32_t width, int32_t height, uint32_t* out);
omr_status oracle_flip_int(const uint32_t* src, uint32_t* dest, int32_t size_x, int32_t size_y,
                           int32_t flip_h, int32_t flip_v);
omr_status oracle_flip_byte(const uint8_t* src, uint8_t* dest, int32_t size_x, int32_t size_y,
                            int32_t flip_h, int32_t flip_v);
omr_status oracle_project_stack(const void* stack, int32_t pixel_type, int32_t big_endian_in,
                                int32_t size_x, int32_t size_y, int32_t size_z, int32_t algorithm,
                                int32_t start, int32_t end, int32_t stepping, void* out,
                                int32_t big_endian_out);
omr_status oracle_mask_indices(const uint8_t* bits, size_t n_bytes, int32_t width,
                               int32_t height, int32_t flip_h, int32_t flip_v, uint8_t* idx);
/* OMR_SEM_* switches (include/omr/omr.h) for every later call; process-wide. */
void oracle_set_semantics(uint32_t flags);
uint32_t oracle_get_semantics(void);
void oracle_jpeg_quant_tables(float quality, uint8_t luma[64], uint8_t chroma[64]);
/* Baseline JPEG (IJG 6b restatement).  Returns bytes written or 0 if cap too small. */
size_t oracle_encode_jpeg(const uint32_t* argb, int32_t width, int32_t height, float quality,
                          uint8_t* out, size_t cap);
/* Quantised coefficients in natural order, MCU order: per MCU Y0 Y1 Y2 Y3 Cb Cr blocks. */
int64_t oracle_jpeg_coefficients(const uint32_t* argb, int32_t width, int32_t height,
                                 float quality, int16_t* coefs, int64_t cap_blocks);
/* Whole reference-CPU request (LUT rebuild + render + flip) over n tiles on n_threads. */
double oracle_render_tiles_mt(const omr_quantum_def* q, const omr_channel_binding* ch,
                              int32_t size_c, const void* const* tile_planes, int32_t n_tiles,
                              int32_t pixel_type, int32_t big_endian, int32_t width,
                              int32_t height, int32_t flip_h, int32_t flip_v, uint32_t* out,
                              int32_t n_threads);

#ifdef __cplusplus
}
#endif
#endif
