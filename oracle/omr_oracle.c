/*
 * omr_oracle.c — CPU restatement of omero-ms-image-region's per-tile rendering path.
 *
 * TEST INFRASTRUCTURE, NOT PRODUCT CODE.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so: as the parity checker and as the
 * timed "reference-CPU proxy".  The product path (libomr.so) never links or calls it.
 *
 * Paths below are relative to src/main/java/com/glencoesoftware/omero/ms/image/region/
 * of the reference (/root/reference).
 *
 * PINNING STATUS
 *   pinned    — flip (ImageRegionRequestHandler.java:616-642, ShapeMaskRequestHandler.java:
 *               128-154): ported index-oracle tests; projection (ProjectionService.java:
 *               176-291): in-repo code restated line for line; mask unpack (:214-221).
 *   pinned    — JPEG: byte-identical entropy-coded data to libjpeg-turbo (the IJG 6b lineage
 *               of the JDK ImageIO writer) at the Java-scaled tables; golden fixtures in
 *               tests/golden/ were produced by PIL (tests/golden/make_golden.py).
 *   UNPINNED  — quantization / codomain / composite arithmetic lives in the un-vendored
 *               omero:server:5.4.10-ice36-b105 (omeis.providers.re.*), absent from this
 *               container (no JVM, no jars, no network).  It is restated
 *               from SURVEY.md Appendix A; every choice sits in the SEMANTICS TABLE below so
 *               it can be corrected in one place.  The GPU kernels implement the same table.
 *
 * SEMANTICS TABLE (Appendix A of SURVEY.md; [H]/[M]/[L] = confidence)
 *   S1 [H] QuantumDef cdStart=0, cdEnd=255, bitResolution=255 (ImageRegionRequestHandler.java:273-277).
 *   S2 [M] family maps f(x,k): linear x; polynomial pow(x,k); logarithmic x>0 ? log(x) : 0
 *          (guard [L]); exponential exp(pow(x,k)).
 *   S3 [M] q(x): x < start -> cdStart; x >= end -> cdEnd; otherwise
 *          v = round(a0*(f(x)-f(start))), a0 = bitRes/(f(end)-f(start));
 *          q = round(a1*v + cdStart) & 0xFF, a1 = (cdEnd-cdStart)/bitRes.  round = Java
 *          Math.round (floor(a+0.5), NaN->0, JDK 8 0.49999999999999994 special case).
 *   S4 [L] noise reduction: x < start+(end-start)/10 -> cdStart; x >= end-(end-start)/10 -> cdEnd.
 *   S5 [M] 8/16-bit integer types quantize through a byte LUT over [globalMin, globalMax]
 *          built per request; a pixel outside that domain is a QuantizationException.
 *          32-bit and float types evaluate q(x) per pixel in double.
 *   S6 [H] reverse intensity: v -> cdEnd - v + cdStart, after quantization (:725-726).
 *   S7 [M] RGB model: channels in index order; contribution (int)(ratio*v) with float
 *          ratio = (c/255f)*(alpha/255f); a .lut channel contributes (R[v],G[v],B[v]);
 *          per-component sum clamped at 255; pixel = 0xFF000000|r<<16|g<<8|b.
 *   S8 [M] greyscale model: first active channel only, (v,v,v); LUTs ignored.  No active
 *          channel renders 0xFF000000.
 *   S9 [H] projection exactly as ProjectionService.java:176-291 (max over [start,end] from 0,
 *          mean/sum over [start,end), double sum, clamp to type max, Java narrowing store).
 *   S10[M] JPEG tables: JPEG.convertToLinearQuality + JPEGQTable.getScaledInstance of the
 *          Annex K luminance and chrominance tables.
 *
 * SWITCHES (oracle_set_semantics; the same OMR_SEM_* flags libomr.so takes per context, so a
 * corrected upstream rule is a one-flag change in both):
 *   OMR_SEM_WINDOW_INT_BOUNDS  S3 for LUT types: x < (int)start -> cdStart, x >= (int)end -> cdEnd.
 *   OMR_SEM_ALPHA_SEPARATE     S7: (int)((int)(c/255f * v) * (alpha/255f)).
 *   OMR_SEM_GREYSCALE_LUT      S8: a .lut channel in greyscale renders (R[v],G[v],B[v]).
 *   OMR_SEM_JPEG_CHROMA_DIV2   S10: chroma base table K2Div2Chrominance = K2.getScaledInstance(0.5f).
 *   OMR_SEM_PROJECTION_ALL_ACTIVE  (libomr.so glue only; the oracle's glue is the tests' loop)
 *   OMR_SEM_LOG_UNGUARDED      S2: logarithmic f(x) = log(x) for every x (NaN below 0, -inf at 0).
 *   OMR_SEM_NOISE_REDUCTION_OFF S4: the noise-reduction flag has no effect.
 *   OMR_SEM_EXP_NORMALIZED     S2: exponential f(x) = exp(pow((x - start)/(end - start), k)).
 *   OMR_SEM_MASK_PIXEL_FLIP    S11: shape mask with width % 8 == 0 flips at pixel level instead of
 *                              reproducing the reference's flip of the still-packed buffer.
 *   S11[H] shape mask (ShapeMaskRequestHandler.java:165-221): MSB-first bit stream; width % 8 != 0
 *          unpacks to a byte per pixel first; flip(bytes, w, h) then runs on whatever buffer it is
 *          given, so with width % 8 == 0 it walks w*h indices of a w*h/8-byte buffer and throws
 *          ArrayIndexOutOfBoundsException -> the future fails -> 404 (ShapeMaskVerticle.java:
 *          119-128).  Every exception inside renderShapeMask is that 404 (OMR_NOT_FOUND).
 */
#include "omr_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ Java numerics */

static int64_t java_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}

static int32_t java_d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return INT32_MAX;
    if (d <= -2147483648.0) return INT32_MIN;
    return (int32_t)d;
}

int64_t oracle_java_round(double a) {
    if (a == 0x1.fffffffffffffp-2) return 0;
    return java_d2l(floor(a + 0.5));
}

static uint32_t g_sem = 0;   /* OMR_SEM_* switches (set before use; not per thread) */

void oracle_set_semantics(uint32_t flags) { g_sem = flags; }
uint32_t oracle_get_semantics(void) { return g_sem; }

/* ------------------------------------------------------------------ quantization (S2-S5) */

/* ws / we: the channel window (OMR_SEM_EXP_NORMALIZED maps x to (x - ws)/(we - ws) first). */
static double family_map(int family, double x, double k, double ws, double we) {
    switch (family) {
    case OMR_FAMILY_POLYNOMIAL: return pow(x, k);
    case OMR_FAMILY_LOGARITHMIC:
        if (g_sem & OMR_SEM_LOG_UNGUARDED) return log(x);
        return x > 0 ? log(x) : 0.0;
    case OMR_FAMILY_EXPONENTIAL:
        if (g_sem & OMR_SEM_EXP_NORMALIZED) return exp(pow((x - ws) / (we - ws), k));
        return exp(pow(x, k));
    default: return x;
    }
}

/* lut_type: the value is an entry of the Quantization_8_16_bit LUT (integer pixel types). */
static int32_t quantize_impl(double x, const omr_channel_binding* cb, const omr_quantum_def* q, int lut_type) {
    const double ws = cb->input_start, we = cb->input_end;
    const int int_bounds = lut_type && (g_sem & OMR_SEM_WINDOW_INT_BOUNDS);
    const double lo = int_bounds ? (double)java_d2i(ws) : ws;
    const double hi = int_bounds ? (double)java_d2i(we) : we;
    if (x < lo) return q->cd_start & 0xFF;
    if (x >= hi) return q->cd_end & 0xFF;
    if (cb->noise_reduction && !(g_sem & OMR_SEM_NOISE_REDUCTION_OFF)) {
        const double dec = (we - ws) / 10.0;
        if (x < ws + dec) return q->cd_start & 0xFF;
        if (x >= we - dec) return q->cd_end & 0xFF;
    }
    const double k = cb->coefficient;
    const double ys = family_map(cb->family, ws, k, ws, we);
    const double ye = family_map(cb->family, we, k, ws, we);
    const double a0 = (double)q->bit_resolution / (ye - ys);
    const double a1 = (double)(q->cd_end - q->cd_start) / (double)q->bit_resolution;
    const double v = (double)oracle_java_round(a0 * (family_map(cb->family, x, k, ws, we) - ys));
    return (int32_t)(oracle_java_round(a1 * v + (double)q->cd_start) & 0xFF);
}

int32_t oracle_quantize(double x, const omr_channel_binding* cb, const omr_quantum_def* q) {
    return quantize_impl(x, cb, q, 0);
}

/* LUT over [globalMin, globalMax] (S5): lut[x - gMin] = q(x). */
omr_status oracle_build_lut(const omr_channel_binding* cb, const omr_quantum_def* q,
                            uint8_t* lut, int64_t n) {
    const int64_t gmin = (int64_t)cb->global_min;
    for (int64_t i = 0; i < n; ++i) lut[i] = (uint8_t)quantize_impl((double)(gmin + i), cb, q, 1);
    return OMR_OK;
}

/* ------------------------------------------------------------------ pixel access */

static int bytes_per_pixel(int t) {
    switch (t) {
    case OMR_PIXELS_INT8: case OMR_PIXELS_UINT8: return 1;
    case OMR_PIXELS_INT16: case OMR_PIXELS_UINT16: return 2;
    case OMR_PIXELS_INT32: case OMR_PIXELS_UINT32: case OMR_PIXELS_FLOAT: return 4;
    case OMR_PIXELS_DOUBLE: return 8;
    default: return 0;
    }
}

static uint64_t load_raw(const uint8_t* p, int nb, int be) {
    uint64_t v = 0;
    if (be) { for (int i = 0; i < nb; ++i) v = (v << 8) | p[i]; }
    else    { for (int i = nb - 1; i >= 0; --i) v = (v << 8) | p[i]; }
    return v;
}

static void store_raw(uint8_t* p, int nb, int be, uint64_t v) {
    if (be) { for (int i = nb - 1; i >= 0; --i) { p[i] = (uint8_t)v; v >>= 8; } }
    else    { for (int i = 0; i < nb; ++i) { p[i] = (uint8_t)v; v >>= 8; } }
}

/* ome.util.PixelData.getPixelValue semantics: signed types sign-extend, unsigned mask. */
static double pixel_value(const uint8_t* p, int t, int be) {
    const uint64_t r = load_raw(p, bytes_per_pixel(t), be);
    switch (t) {
    case OMR_PIXELS_INT8: return (double)(int8_t)r;
    case OMR_PIXELS_UINT8: return (double)(uint8_t)r;
    case OMR_PIXELS_INT16: return (double)(int16_t)r;
    case OMR_PIXELS_UINT16: return (double)(uint16_t)r;
    case OMR_PIXELS_INT32: return (double)(int32_t)r;
    case OMR_PIXELS_UINT32: return (double)(uint32_t)r;
    case OMR_PIXELS_FLOAT: { uint32_t u = (uint32_t)r; float f; memcpy(&f, &u, 4); return f; }
    case OMR_PIXELS_DOUBLE: { double d; memcpy(&d, &r, 8); return d; }
    }
    return 0;
}

static int is_lut_type(int t) { return bytes_per_pixel(t) <= 2; }

static void type_range(int t, double* lo, double* hi) {
    switch (t) {
    case OMR_PIXELS_INT8: *lo = -128; *hi = 127; break;
    case OMR_PIXELS_UINT8: *lo = 0; *hi = 255; break;
    case OMR_PIXELS_INT16: *lo = -32768; *hi = 32767; break;
    case OMR_PIXELS_UINT16: *lo = 0; *hi = 65535; break;
    default: *lo = 0; *hi = 0; break;
    }
}

/* ------------------------------------------------------------------ render (S5-S8) */

typedef struct {
    int active;
    uint8_t* lut;      /* per-request LUT for <=16-bit types */
    int64_t gmin, gmax;
    float ratio[3];    /* (c/255f)*(alpha/255f) */
    float cratio[3];   /* c/255f */
    float alpha;       /* alpha/255f */
} chan_state;

omr_status oracle_render_packed_int(const omr_quantum_def* q, const omr_channel_binding* ch,
                                    int32_t size_c, const void* const* planes,
                                    int64_t row_stride, int32_t pixel_type, int32_t big_endian,
                                    int32_t width, int32_t height, uint32_t* out) {
    const int nb = bytes_per_pixel(pixel_type);
    if (!nb || size_c < 0 || width < 0 || height < 0 || !q || (size_c && !ch)) return OMR_INVALID_ARGUMENT;
    if (row_stride == 0) row_stride = width;
    chan_state* st = (chan_state*)calloc(size_c > 0 ? size_c : 1, sizeof(chan_state));
    omr_status rc = OMR_OK;
    int first_active = -1;
    for (int c = 0; c < size_c; ++c) {
        st[c].active = ch[c].active != 0;
        if (!st[c].active) continue;
        if (!planes || !planes[c]) { rc = OMR_INVALID_ARGUMENT; goto done; }
        if (first_active < 0) first_active = c;
        if (is_lut_type(pixel_type)) {
            double lo, hi;
            type_range(pixel_type, &lo, &hi);
            st[c].gmin = (int64_t)ch[c].global_min;
            st[c].gmax = (int64_t)ch[c].global_max;
            if (st[c].gmax < st[c].gmin) { rc = OMR_INVALID_ARGUMENT; goto done; }
            const int64_t n = st[c].gmax - st[c].gmin + 1;
            st[c].lut = (uint8_t*)malloc((size_t)n);
            oracle_build_lut(&ch[c], q, st[c].lut, n);
        }
        const float alpha = (float)ch[c].rgba[3] / 255.0f;
        st[c].alpha = alpha;
        for (int k = 0; k < 3; ++k) {
            st[c].cratio[k] = (float)ch[c].rgba[k] / 255.0f;
            st[c].ratio[k] = st[c].cratio[k] * alpha;
        }
    }
    for (int y = 0; y < height; ++y) {
        for (int x = 0; x < width; ++x) {
            int r = 0, g = 0, b = 0;
            for (int c = 0; c < size_c; ++c) {
                if (!st[c].active) continue;
                if (q->model == OMR_MODEL_GREYSCALE && c != first_active) continue;
                const uint8_t* p = (const uint8_t*)planes[c] + ((int64_t)y * row_stride + x) * nb;
                const double xv = pixel_value(p, pixel_type, big_endian);
                int v;
                if (st[c].lut) {
                    const int64_t xi = (int64_t)xv;
                    if (xi < st[c].gmin || xi > st[c].gmax) { rc = OMR_QUANTIZATION; goto done; }
                    v = st[c].lut[xi - st[c].gmin];
                } else {
                    v = oracle_quantize(xv, &ch[c], q);
                }
                if (ch[c].reverse) v = (q->cd_end - v + q->cd_start) & 0xFF;
                if (q->model == OMR_MODEL_GREYSCALE) {
                    if (ch[c].lut && (g_sem & OMR_SEM_GREYSCALE_LUT)) {
                        r = ch[c].lut[v]; g = ch[c].lut[256 + v]; b = ch[c].lut[512 + v];
                    } else {
                        r = g = b = v;
                    }
                    break;
                }
                int cr, cg, cb;
                if (ch[c].lut) {
                    cr = ch[c].lut[v]; cg = ch[c].lut[256 + v]; cb = ch[c].lut[512 + v];
                } else if (g_sem & OMR_SEM_ALPHA_SEPARATE) {
                    cr = (int)((float)(int)(st[c].cratio[0] * (float)v) * st[c].alpha);
                    cg = (int)((float)(int)(st[c].cratio[1] * (float)v) * st[c].alpha);
                    cb = (int)((float)(int)(st[c].cratio[2] * (float)v) * st[c].alpha);
                } else {
                    cr = (int)(st[c].ratio[0] * (float)v);
                    cg = (int)(st[c].ratio[1] * (float)v);
                    cb = (int)(st[c].ratio[2] * (float)v);
                }
                r += cr; if (r > 255) r = 255;
                g += cg; if (g > 255) g = 255;
                b += cb; if (b > 255) b = 255;
            }
            out[(int64_t)y * width + x] = 0xFF000000u | ((uint32_t)r << 16) | ((uint32_t)g << 8) | (uint32_t)b;
        }
    }
done:
    for (int c = 0; c < size_c; ++c) free(st[c].lut);
    free(st);
    return rc;
}

/* ------------------------------------------------------------------ flips */
/* ImageRegionRequestHandler.flip (:616-642): dest[|(yo-y-1)*w| + |xo-x-1|] = src[y*w+x]. */
omr_status oracle_flip_int(const uint32_t* src, uint32_t* dest, int32_t size_x, int32_t size_y,
                           int32_t flip_h, int32_t flip_v) {
    if (!flip_h && !flip_v) {
        if (src && dest && size_x > 0 && size_y > 0) memcpy(dest, src, (size_t)size_x * size_y * 4);
        return OMR_OK;
    }
    if (!src) return OMR_INVALID_ARGUMENT;
    if (size_x == 0 || size_y == 0) return OMR_INVALID_ARGUMENT;
    const int64_t xo = flip_h ? size_x : 1, yo = flip_v ? size_y : 1;
    for (int64_t x = 0; x < size_x; ++x)
        for (int64_t y = 0; y < size_y; ++y)
            dest[llabs((yo - y - 1) * size_x) + llabs(xo - x - 1)] = src[y * size_x + x];
    return OMR_OK;
}

omr_status oracle_flip_byte(const uint8_t* src, uint8_t* dest, int32_t size_x, int32_t size_y,
                            int32_t flip_h, int32_t flip_v) {
    if (!flip_h && !flip_v) {
        if (src && dest && size_x > 0 && size_y > 0) memcpy(dest, src, (size_t)size_x * size_y);
        return OMR_OK;
    }
    if (!src) return OMR_INVALID_ARGUMENT;
    if (size_x == 0 || size_y == 0) return OMR_INVALID_ARGUMENT;
    const int64_t xo = flip_h ? size_x : 1, yo = flip_v ? size_y : 1;
    for (int64_t x = 0; x < size_x; ++x)
        for (int64_t y = 0; y < size_y; ++y)
            dest[llabs((yo - y - 1) * size_x) + llabs(xo - x - 1)] = src[y * size_x + x];
    return OMR_OK;
}

/* ------------------------------------------------------------------ projection (S9) */

static double type_maximum(int t) {  /* ome.util.PixelData.getMaximum() */
    switch (t) {
    case OMR_PIXELS_INT8: return 127.0;
    case OMR_PIXELS_UINT8: return 255.0;
    case OMR_PIXELS_INT16: return 32767.0;
    case OMR_PIXELS_UINT16: return 65535.0;
    case OMR_PIXELS_INT32: return 2147483647.0;
    case OMR_PIXELS_UINT32: return 4294967295.0;
    case OMR_PIXELS_FLOAT: return 3.4028234663852886e38;
    default: return 1.7976931348623157e308;
    }
}

/* PixelData.setPixelValue(i, double): Java narrowing casts into a ByteBuffer. */
static void set_pixel_value(uint8_t* p, int t, int be, double v) {
    const int nb = bytes_per_pixel(t);
    uint64_t raw = 0;
    switch (t) {
    case OMR_PIXELS_INT8: case OMR_PIXELS_UINT8: raw = (uint8_t)(int8_t)java_d2i(v); break;
    case OMR_PIXELS_INT16: case OMR_PIXELS_UINT16: raw = (uint16_t)(int16_t)java_d2i(v); break;
    case OMR_PIXELS_INT32: raw = (uint32_t)java_d2i(v); break;
    case OMR_PIXELS_UINT32: raw = (uint32_t)java_d2l(v); break;
    case OMR_PIXELS_FLOAT: { float f = (float)v; uint32_t u; memcpy(&u, &f, 4); raw = u; break; }
    case OMR_PIXELS_DOUBLE: memcpy(&raw, &v, 8); break;
    }
    store_raw(p, nb, be, raw);
}

omr_status oracle_project_stack(const void* stack, int32_t pixel_type, int32_t big_endian_in,
                                int32_t size_x, int32_t size_y, int32_t size_z, int32_t algorithm,
                                int32_t start, int32_t end, int32_t stepping, void* out,
                                int32_t big_endian_out) {
    const int nb = bytes_per_pixel(pixel_type);
    if (!nb) return OMR_INVALID_ARGUMENT;
    /* zIntervalBoundsCheck (ProjectionService.java:154-161), outOfBoundsStepping (:140-144) */
    if (start < 0 || end < 0) return OMR_INVALID_ARGUMENT;
    if (start >= size_z || end >= size_z) return OMR_INVALID_ARGUMENT;
    if (stepping <= 0) return OMR_INVALID_ARGUMENT;
    if (algorithm < OMR_PROJECTION_MAX || algorithm > OMR_PROJECTION_SUM) return OMR_INVALID_ARGUMENT;
    const int64_t plane = (int64_t)size_x * size_y;
    const uint8_t* from = (const uint8_t*)stack;
    uint8_t* to = (uint8_t*)out;
    const double plane_max = type_maximum(pixel_type);
    for (int64_t i = 0; i < plane; ++i) {
        double pv = 0;
        if (algorithm == OMR_PROJECTION_MAX) {       /* :182-196 */
            for (int z = start; z <= end; z += stepping) {
                const double sv = pixel_value(from + (plane * z + i) * nb, pixel_type, big_endian_in);
                if (sv > pv) pv = sv;
            }
        } else {                                      /* :268-288 */
            int count = 0;
            for (int z = start; z < end; z += stepping) {
                pv += pixel_value(from + (plane * z + i) * nb, pixel_type, big_endian_in);
                count++;
            }
            if (algorithm == OMR_PROJECTION_MEAN) pv = pv / count;
            if (pv > plane_max) pv = plane_max;
        }
        set_pixel_value(to + i * nb, pixel_type, big_endian_out, pv);
    }
    return OMR_OK;
}

/* ------------------------------------------------------------------ shape mask (S11) */
/* ShapeMaskRequestHandler.java:165-221 -> 0/1 palette index per pixel.  OMR_NOT_FOUND is every
 * exception the reference raises there (404 via ShapeMaskVerticle.java:119-128). */
omr_status oracle_mask_indices(const uint8_t* bits, size_t n_bytes, int32_t width,
                               int32_t height, int32_t flip_h, int32_t flip_v, uint8_t* idx) {
    if (width <= 0 || height <= 0 || !bits) return OMR_NOT_FOUND;      /* IAE / NPE */
    const int64_t n = (int64_t)width * height;
    if (n > INT32_MAX) return OMR_NOT_FOUND;                            /* Java int w*h wraps */
    if ((int64_t)n_bytes * 8 < n) return OMR_NOT_FOUND;                 /* IOOBE / RasterFormatException */
    const int flip = flip_h || flip_v;
    if (width % 8 == 0 && flip && !(g_sem & OMR_SEM_MASK_PIXEL_FLIP)) {
        /* :179-181 flips the packed buffer: flip(bytes, w, h) reads and writes w*h byte indices */
        if ((int64_t)n_bytes < n) return OMR_NOT_FOUND;                 /* ArrayIndexOutOfBounds */
        uint8_t* dest = (uint8_t*)calloc(n_bytes, 1);                   /* new byte[src.length] */
        oracle_flip_byte(bits, dest, width, height, flip_h, flip_v);
        for (int64_t i = 0; i < n; ++i) idx[i] = (dest[i >> 3] >> (7 - (i & 7))) & 1;
        free(dest);
        return OMR_OK;
    }
    uint8_t* tmp = (uint8_t*)malloc((size_t)n);
    for (int64_t i = 0; i < n; ++i) tmp[i] = (bits[i >> 3] >> (7 - (i & 7))) & 1;
    omr_status rc = oracle_flip_byte(tmp, idx, width, height, flip_h, flip_v);
    if (!flip) memcpy(idx, tmp, (size_t)n);
    free(tmp);
    return rc;
}

/* ------------------------------------------------------------------ JPEG (IJG 6b restatement) */

static const int kStdLuma[64] = {
    16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
    14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
    18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
static const int kStdChroma[64] = {
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
static const int kZigzag[64] = {
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

static const uint8_t kBitsDcL[17] = {0, 0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
static const uint8_t kValDc[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
static const uint8_t kBitsDcC[17] = {0, 0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
static const uint8_t kBitsAcL[17] = {0, 0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
static const uint8_t kValAcL[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07,
    0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0,
    0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28,
    0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49,
    0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69,
    0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89,
    0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5,
    0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa};
static const uint8_t kBitsAcC[17] = {0, 0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
static const uint8_t kValAcC[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71,
    0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0,
    0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26,
    0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48,
    0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68,
    0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86, 0x87,
    0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5,
    0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa};

/* JPEGQTable.getScaledInstance(scale, true): (int)(q*scale + 0.5f) clamped to [1, 255]. */
static int qscale(int qv, float scale) {
    volatile float a = (float)qv * scale;
    const int sv = (int)(a + 0.5f);
    return sv < 1 ? 1 : sv > 255 ? 255 : sv;
}

/* javax.imageio JPEG.convertToLinearQuality + JPEGQTable.getScaledInstance(scale, true) (S10). */
void oracle_jpeg_quant_tables(float quality, uint8_t luma[64], uint8_t chroma[64]) {
    float qf = quality;
    if (qf <= 0.0f) qf = 0.01f;
    if (qf > 1.00f) qf = 1.00f;
    if (qf < 0.5f) qf = 0.5f / qf;
    else qf = 2.0f - (qf * 2.0f);
    for (int i = 0; i < 64; ++i) {
        luma[i] = (uint8_t)qscale(kStdLuma[i], qf);
        const int cbase = (g_sem & OMR_SEM_JPEG_CHROMA_DIV2) ? qscale(kStdChroma[i], 0.5f) : kStdChroma[i];
        chroma[i] = (uint8_t)qscale(cbase, qf);
    }
}

/* jfdctint.c (IJG 6b) — islow forward DCT, in place on 64 ints. */
#define CONST_BITS 13
#define PASS1_BITS 2
#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))
static void fdct_islow(int* d) {
    for (int pass = 0; pass < 2; ++pass) {
        const int step = pass ? 8 : 1, stride = pass ? 1 : 8;
        for (int r = 0; r < 8; ++r) {
            int* p = d + r * stride;
            int32_t tmp0 = p[0 * step] + p[7 * step], tmp7 = p[0 * step] - p[7 * step];
            int32_t tmp1 = p[1 * step] + p[6 * step], tmp6 = p[1 * step] - p[6 * step];
            int32_t tmp2 = p[2 * step] + p[5 * step], tmp5 = p[2 * step] - p[5 * step];
            int32_t tmp3 = p[3 * step] + p[4 * step], tmp4 = p[3 * step] - p[4 * step];
            int32_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3;
            int32_t tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
            const int sh = pass ? CONST_BITS + PASS1_BITS : CONST_BITS - PASS1_BITS;
            if (pass) {
                p[0 * step] = DESCALE(tmp10 + tmp11, PASS1_BITS);
                p[4 * step] = DESCALE(tmp10 - tmp11, PASS1_BITS);
            } else {
                p[0 * step] = (tmp10 + tmp11) << PASS1_BITS;
                p[4 * step] = (tmp10 - tmp11) << PASS1_BITS;
            }
            int32_t z1 = (tmp12 + tmp13) * 4433;
            p[2 * step] = DESCALE(z1 + tmp13 * 6270, sh);
            p[6 * step] = DESCALE(z1 + tmp12 * (-15137), sh);
            z1 = tmp4 + tmp7;
            int32_t z2 = tmp5 + tmp6, z3 = tmp4 + tmp6, z4 = tmp5 + tmp7;
            int32_t z5 = (z3 + z4) * 9633;
            tmp4 = tmp4 * 2446; tmp5 = tmp5 * 16819; tmp6 = tmp6 * 25172; tmp7 = tmp7 * 12299;
            z1 = z1 * (-7373); z2 = z2 * (-20995); z3 = z3 * (-16069); z4 = z4 * (-3196);
            z3 += z5; z4 += z5;
            p[7 * step] = DESCALE(tmp4 + z1 + z3, sh);
            p[5 * step] = DESCALE(tmp5 + z2 + z4, sh);
            p[3 * step] = DESCALE(tmp6 + z2 + z3, sh);
            p[1 * step] = DESCALE(tmp7 + z1 + z4, sh);
        }
    }
}

/* jcdctmgr.c forward_DCT quantisation: divisor = q << 3, sign-symmetric rounding. */
static int16_t quantize_coef(int32_t t, int qval) {
    const int32_t div = qval << 3;
    if (t < 0) { t = -t; t += div >> 1; t = t >= div ? t / div : 0; return (int16_t)-t; }
    t += div >> 1;
    return (int16_t)(t >= div ? t / div : 0);
}

/* Component planes after jccolor/jcprepct/jcsample (IJG edge replication). */
typedef struct {
    int w, h;          /* padded plane dims in samples */
    uint8_t* s;
} jplane;

static void jpeg_planes(const uint32_t* argb, int W, int H, jplane* Y, jplane* Cb, jplane* Cr) {
    /* jccolor.c rgb_ycc_convert: 16-bit fixed point tables */
#define FIXJ(x) ((int32_t)((x) * 65536.0 + 0.5))
    const int32_t ONE_HALF = 1 << 15, CBCR_OFF = 128 << 16;
    const int mcux = (W + 15) / 16, mcuy = (H + 15) / 16;
    const int Hev = H + (H & 1);                 /* jcprepct: colour buffer padded to max_v_samp rows */
    const int yw = ((W + 7) / 8) * 8, yh = mcuy * 16;
    const int cw = mcux * 8, ch = mcuy * 8;
    Y->w = yw; Y->h = yh; Y->s = (uint8_t*)malloc((size_t)yw * yh);
    Cb->w = cw; Cb->h = ch; Cb->s = (uint8_t*)malloc((size_t)cw * ch);
    Cr->w = cw; Cr->h = ch; Cr->s = (uint8_t*)malloc((size_t)cw * ch);
    const int fw = cw * 2;                       /* h2v2 input expanded to output_cols*2 */
    uint8_t* fcb = (uint8_t*)malloc((size_t)fw * Hev);
    uint8_t* fcr = (uint8_t*)malloc((size_t)fw * Hev);
    for (int y = 0; y < Hev; ++y) {
        const int sy = y < H ? y : H - 1;
        for (int x = 0; x < (fw > yw ? fw : yw); ++x) {
            const int sx = x < W ? x : W - 1;
            const uint32_t p = argb[(int64_t)sy * W + sx];
            const int r = (p >> 16) & 0xFF, g = (p >> 8) & 0xFF, b = p & 0xFF;
            const int yy = (int)((FIXJ(0.29900) * r + FIXJ(0.58700) * g + FIXJ(0.11400) * b + ONE_HALF) >> 16);
            const int cb = (int)((-FIXJ(0.16874) * r - FIXJ(0.33126) * g + FIXJ(0.50000) * b + CBCR_OFF + ONE_HALF - 1) >> 16);
            const int cr = (int)((FIXJ(0.50000) * r - FIXJ(0.41869) * g - FIXJ(0.08131) * b + CBCR_OFF + ONE_HALF - 1) >> 16);
            if (x < yw) Y->s[(int64_t)y * yw + x] = (uint8_t)yy;
            if (x < fw) { fcb[(int64_t)y * fw + x] = (uint8_t)cb; fcr[(int64_t)y * fw + x] = (uint8_t)cr; }
        }
    }
    for (int y = Hev; y < yh; ++y) memcpy(Y->s + (int64_t)y * yw, Y->s + (int64_t)(Hev - 1) * yw, yw);
    const int chv = Hev / 2;                     /* downsampled rows produced from real data */
    for (int y = 0; y < ch; ++y) {
        const int sy = y < chv ? y : chv - 1;
        for (int x = 0; x < cw; ++x) {
            if (y >= chv) { Cb->s[y * cw + x] = Cb->s[sy * cw + x]; Cr->s[y * cw + x] = Cr->s[sy * cw + x]; continue; }
            const int bias = (x & 1) ? 2 : 1;    /* jcsample.c h2v2_downsample bias 1,2,1,2,... */
            const uint8_t* a0 = fcb + (int64_t)(2 * y) * fw + 2 * x;
            const uint8_t* a1 = a0 + fw;
            Cb->s[y * cw + x] = (uint8_t)((a0[0] + a0[1] + a1[0] + a1[1] + bias) >> 2);
            const uint8_t* b0 = fcr + (int64_t)(2 * y) * fw + 2 * x;
            const uint8_t* b1 = b0 + fw;
            Cr->s[y * cw + x] = (uint8_t)((b0[0] + b0[1] + b1[0] + b1[1] + bias) >> 2);
        }
    }
    free(fcb);
    free(fcr);
#undef FIXJ
}

static void block_coefs(const jplane* P, int bx, int by, const uint8_t* qt, int16_t* out) {
    int d[64];
    for (int r = 0; r < 8; ++r)
        for (int c = 0; c < 8; ++c) d[r * 8 + c] = (int)P->s[(int64_t)(by * 8 + r) * P->w + bx * 8 + c] - 128;
    fdct_islow(d);
    for (int i = 0; i < 64; ++i) out[i] = quantize_coef(d[i], qt[i]);
}

/* jccoefct.c compress_data: MCU order with right/bottom dummy blocks (DC copied, AC zero). */
int64_t oracle_jpeg_coefficients(const uint32_t* argb, int32_t width, int32_t height,
                                 float quality, int16_t* coefs, int64_t cap_blocks) {
    if (width <= 0 || height <= 0) return -1;
    uint8_t ql[64], qc[64];
    oracle_jpeg_quant_tables(quality, ql, qc);
    jplane Y, Cb, Cr;
    jpeg_planes(argb, width, height, &Y, &Cb, &Cr);
    const int mcux = (width + 15) / 16, mcuy = (height + 15) / 16;
    const int ywib = (width + 7) / 8, yhib = (height + 7) / 8;
    const int64_t nblocks = (int64_t)mcux * mcuy * 6;
    if (nblocks > cap_blocks) { free(Y.s); free(Cb.s); free(Cr.s); return -nblocks; }
    int64_t blk = 0;
    for (int my = 0; my < mcuy; ++my) {
        for (int mx = 0; mx < mcux; ++mx) {
            int16_t* mcu = coefs + blk * 64;
            for (int yi = 0; yi < 2; ++yi) {
                for (int xi = 0; xi < 2; ++xi) {
                    int16_t* o = mcu + (yi * 2 + xi) * 64;
                    const int bx = mx * 2 + xi, by = my * 2 + yi;
                    if (by >= yhib) {          /* bottom dummy row: DC of MCU_buffer[blkn-1] */
                        memset(o, 0, 64 * 2);
                        o[0] = mcu[(yi * 2 - 1) * 64];
                    } else if (bx >= ywib) {   /* right dummy: DC of left neighbour */
                        memset(o, 0, 64 * 2);
                        o[0] = o[-64];
                    } else {
                        block_coefs(&Y, bx, by, ql, o);
                    }
                }
            }
            block_coefs(&Cb, mx, my, qc, mcu + 4 * 64);
            block_coefs(&Cr, mx, my, qc, mcu + 5 * 64);
            blk += 6;
        }
    }
    free(Y.s); free(Cb.s); free(Cr.s);
    return nblocks;
}

typedef struct { uint16_t code[256]; uint8_t size[256]; } hufftab;

static void make_huff(const uint8_t* bits, const uint8_t* vals, hufftab* t) {
    memset(t, 0, sizeof(*t));
    int k = 0; unsigned code = 0;
    for (int l = 1; l <= 16; ++l) {
        for (int i = 0; i < bits[l]; ++i) { t->code[vals[k]] = (uint16_t)code; t->size[vals[k]] = (uint8_t)l; ++k; ++code; }
        code <<= 1;
    }
}

typedef struct { uint8_t* out; size_t cap, len; uint32_t acc; int nbits; int overflow; } bitw;

static void put_byte(bitw* w, uint8_t b) {
    if (w->len < w->cap) w->out[w->len++] = b; else w->overflow = 1;
}
static void put_bits(bitw* w, uint32_t v, int n) {
    for (int i = n - 1; i >= 0; --i) {
        w->acc = (w->acc << 1) | ((v >> i) & 1);
        if (++w->nbits == 8) {
            const uint8_t b = (uint8_t)w->acc;
            put_byte(w, b);
            if (b == 0xFF) put_byte(w, 0);
            w->acc = 0; w->nbits = 0;
        }
    }
}

static void encode_block(bitw* w, const int16_t* blk, int* last_dc, const hufftab* dc, const hufftab* ac) {
    int temp = blk[0] - *last_dc, temp2 = temp;
    *last_dc = blk[0];
    if (temp < 0) { temp = -temp; temp2--; }
    int nbits = 0;
    while (temp) { nbits++; temp >>= 1; }
    put_bits(w, dc->code[nbits], dc->size[nbits]);
    if (nbits) put_bits(w, (uint32_t)temp2 & ((1u << nbits) - 1), nbits);
    int r = 0;
    for (int k = 1; k < 64; ++k) {
        temp = blk[kZigzag[k]];
        if (temp == 0) { r++; continue; }
        while (r > 15) { put_bits(w, ac->code[0xF0], ac->size[0xF0]); r -= 16; }
        temp2 = temp;
        if (temp < 0) { temp = -temp; temp2--; }
        nbits = 1;
        while ((temp >>= 1)) nbits++;
        const int i = (r << 4) + nbits;
        put_bits(w, ac->code[i], ac->size[i]);
        put_bits(w, (uint32_t)temp2 & ((1u << nbits) - 1), nbits);
        r = 0;
    }
    if (r > 0) put_bits(w, ac->code[0], ac->size[0]);
}

static void put_marker_dht(bitw* w, int cls_id, const uint8_t* bits, const uint8_t* vals) {
    int n = 0;
    for (int i = 1; i <= 16; ++i) n += bits[i];
    put_byte(w, 0xFF); put_byte(w, 0xC4);
    put_byte(w, (uint8_t)((2 + 1 + 16 + n) >> 8)); put_byte(w, (uint8_t)(2 + 1 + 16 + n));
    put_byte(w, (uint8_t)cls_id);
    for (int i = 1; i <= 16; ++i) put_byte(w, bits[i]);
    for (int i = 0; i < n; ++i) put_byte(w, vals[i]);
}

size_t oracle_encode_jpeg(const uint32_t* argb, int32_t width, int32_t height, float quality,
                          uint8_t* out, size_t cap) {
    if (width <= 0 || height <= 0 || width > 65535 || height > 65535) return 0;
    const int mcux = (width + 15) / 16, mcuy = (height + 15) / 16;
    const int64_t nblocks = (int64_t)mcux * mcuy * 6;
    int16_t* coefs = (int16_t*)malloc((size_t)nblocks * 64 * 2);
    oracle_jpeg_coefficients(argb, width, height, quality, coefs, nblocks);
    uint8_t ql[64], qc[64];
    oracle_jpeg_quant_tables(quality, ql, qc);
    bitw w = {out, cap, 0, 0, 0, 0};
    static const uint8_t hdr[] = {0xFF, 0xD8, 0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0x00,
                                  0x01, 0x01, 0x00, 0x00, 0x01, 0x00, 0x01, 0x00, 0x00};
    for (size_t i = 0; i < sizeof(hdr); ++i) put_byte(&w, hdr[i]);
    for (int t = 0; t < 2; ++t) {
        put_byte(&w, 0xFF); put_byte(&w, 0xDB); put_byte(&w, 0); put_byte(&w, 67); put_byte(&w, (uint8_t)t);
        for (int i = 0; i < 64; ++i) put_byte(&w, (t ? qc : ql)[kZigzag[i]]);
    }
    const uint8_t sof[] = {0xFF, 0xC0, 0, 17, 8, (uint8_t)(height >> 8), (uint8_t)height,
                           (uint8_t)(width >> 8), (uint8_t)width, 3, 1, 0x22, 0, 2, 0x11, 1, 3, 0x11, 1};
    for (size_t i = 0; i < sizeof(sof); ++i) put_byte(&w, sof[i]);
    put_marker_dht(&w, 0x00, kBitsDcL, kValDc);
    put_marker_dht(&w, 0x10, kBitsAcL, kValAcL);
    put_marker_dht(&w, 0x01, kBitsDcC, kValDc);
    put_marker_dht(&w, 0x11, kBitsAcC, kValAcC);
    static const uint8_t sos[] = {0xFF, 0xDA, 0, 12, 3, 1, 0x00, 2, 0x11, 3, 0x11, 0, 63, 0};
    for (size_t i = 0; i < sizeof(sos); ++i) put_byte(&w, sos[i]);
    hufftab dcl, acl, dcc, acc;
    make_huff(kBitsDcL, kValDc, &dcl); make_huff(kBitsAcL, kValAcL, &acl);
    make_huff(kBitsDcC, kValDc, &dcc); make_huff(kBitsAcC, kValAcC, &acc);
    int dc[3] = {0, 0, 0};
    for (int64_t m = 0; m < nblocks / 6; ++m) {
        const int16_t* mcu = coefs + m * 6 * 64;
        for (int b = 0; b < 4; ++b) encode_block(&w, mcu + b * 64, &dc[0], &dcl, &acl);
        encode_block(&w, mcu + 4 * 64, &dc[1], &dcc, &acc);
        encode_block(&w, mcu + 5 * 64, &dc[2], &dcc, &acc);
    }
    if (w.nbits) put_bits(&w, 0x7F, 8 - w.nbits);   /* jchuff.c flush_bits: pad with 1s */
    put_byte(&w, 0xFF); put_byte(&w, 0xD9);
    free(coefs);
    return w.overflow ? 0 : w.len;
}

/* ------------------------------------------------------------------ CPU baseline */
/* The reference's per-request work (new Renderer + LUT rebuild per request,
 * ImageRegionRequestHandler.java:436-440; render; flip) over a pool of worker threads,
 * mirroring the Vert.x worker-verticle request parallelism (ImageRegionMicroserviceVerticle.java:149-165). */
typedef struct {
    const omr_quantum_def* q; const omr_channel_binding* ch; int size_c;
    const void* const* tile_planes; int n_tiles; int pixel_type, be, w, h, fh, fv;
    uint32_t* out; int next; pthread_mutex_t mu; uint32_t* scratch_unused;
} mt_job;

static void* mt_worker(void* arg) {
    mt_job* j = (mt_job*)arg;
    const int64_t n = (int64_t)j->w * j->h;
    uint32_t* tmp = (uint32_t*)malloc((size_t)n * 4);
    uint32_t* tmp2 = (uint32_t*)malloc((size_t)n * 4);
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const int t = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (t >= j->n_tiles) break;
        uint32_t* dst = j->out ? j->out + (int64_t)t * n : tmp;   /* NULL out: per-thread scratch */
        if ((j->fh || j->fv) && j->out) {
            oracle_render_packed_int(j->q, j->ch, j->size_c, j->tile_planes + (int64_t)t * j->size_c, 0,
                                     j->pixel_type, j->be, j->w, j->h, tmp);
            oracle_flip_int(tmp, dst, j->w, j->h, j->fh, j->fv);
        } else if (j->fh || j->fv) {
            oracle_render_packed_int(j->q, j->ch, j->size_c, j->tile_planes + (int64_t)t * j->size_c, 0,
                                     j->pixel_type, j->be, j->w, j->h, tmp);
            oracle_flip_int(tmp, tmp2, j->w, j->h, j->fh, j->fv);
        } else {
            oracle_render_packed_int(j->q, j->ch, j->size_c, j->tile_planes + (int64_t)t * j->size_c, 0,
                                     j->pixel_type, j->be, j->w, j->h, dst);
        }
    }
    free(tmp);
    free(tmp2);
    return NULL;
}

double oracle_render_tiles_mt(const omr_quantum_def* q, const omr_channel_binding* ch,
                              int32_t size_c, const void* const* tile_planes, int32_t n_tiles,
                              int32_t pixel_type, int32_t big_endian, int32_t width,
                              int32_t height, int32_t flip_h, int32_t flip_v, uint32_t* out,
                              int32_t n_threads) {
    mt_job j = {q, ch, size_c, tile_planes, n_tiles, pixel_type, big_endian, width, height,
                flip_h, flip_v, out, 0, PTHREAD_MUTEX_INITIALIZER, NULL};
    if (n_threads < 1) n_threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < n_threads; ++i) pthread_create(&th[i], NULL, mt_worker, &j);
    for (int i = 0; i < n_threads; ++i) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
