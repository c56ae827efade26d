/*
 * omr_jni.c — JNI shim between the reference's Java host code and libomr.so (include/omr/omr.h).
 *
 * Java side: java/src/main/java/com/glencoesoftware/omero/ms/image/region/gpu/OmrNative.java.
 * Build (needs a JDK, absent from this image — see jni/Makefile and INTEGRATION.md §3):
 *   make -C jni JAVA_HOME=/usr/lib/jvm/java-8-openjdk-amd64
 * Tests: tests/jni/ compiles this file against a mock JVM (a test-only jni.h with the JNI function
 * table in specification order, mock_jni.c behind it) and tests/test_jni_shim*.py drive every
 * native method through it, against the CPU restatement.
 *
 * Call sites it serves (paths relative to src/main/java/com/glencoesoftware/omero/ms/image/region/):
 *   renderPackedInt     renderer.renderAsPackedInt + flip      ImageRegionRequestHandler.java:559, :574-575
 *   projectStack        projectionService.projectStack         ProjectionService.java:46-120
 *   encodeJpeg          compressionService.compressToStream     ImageRegionRequestHandler.java:576-582
 *   encodePng/Tiff      ImageIO.write / TIFFImageWriter         ImageRegionRequestHandler.java:583-600
 *   renderShapeMaskPng  renderShapeMask(Color, byte[], w, h)    ShapeMaskRequestHandler.java:165-207
 *   batcher* / pool*    one Renderer per request on each worker ImageRegionMicroserviceVerticle.java:149-165
 *   *SubmitProjected    the projection glue of render           ImageRegionRequestHandler.java:506-558
 *   *SubmitMask         renderShapeMask per worker              ShapeMaskVerticle.java:121-149
 *
 * Rules kept here:
 *  - every array length is checked (64-bit arithmetic) before any pixel byte moves; a short or
 *    null array is OmrException(INVALID_ARGUMENT), never a read or write past a Java array;
 *  - no critical array is held across a GPU call: pixels are copied with Get<T>ArrayRegion into
 *    the context's pinned staging and results written back with Set<T>ArrayRegion, so the GC is
 *    never blocked by a render;
 *  - every local reference taken in a loop is deleted in that loop;
 *  - after any JNI call that can throw, a pending exception returns at once;
 *  - library failures become OmrException(status, message); the status maps to the reference's
 *    HTTP outcome (omr.h).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "omr/omr.h"

#define PKG "com/glencoesoftware/omero/ms/image/region/gpu/"
#define NCH_FIELDS 13          /* doubles per channel in the packed settings array (OmrNative.java) */
#define MAX_CH OMR_MAX_REQUEST_CHANNELS

/* The handle Java holds for a context: the library context plus a grow-only pinned staging
 * buffer the pixels travel through (omr_pinned_alloc: page-locked, so the H2D / D2H copies run
 * at full PCIe rate and nothing pageable is touched by the DMA engines). */
typedef struct {
    omr_ctx* ctx;
    uint8_t* pin;
    size_t pin_cap;
} jctx;

static void throw_omr(JNIEnv* env, jint status, const char* msg) {
    if ((*env)->ExceptionCheck(env)) return;            /* keep the first exception */
    jclass cls = (*env)->FindClass(env, PKG "OmrException");
    if (!cls) return;                                   /* NoClassDefFoundError already pending */
    jmethodID ctor = (*env)->GetMethodID(env, cls, "<init>", "(ILjava/lang/String;)V");
    if (!ctor) return;
    jstring jmsg = (*env)->NewStringUTF(env, msg ? msg : "");
    if (!jmsg) return;
    jobject ex = (*env)->NewObject(env, cls, ctor, status, jmsg);
    if (ex) (*env)->Throw(env, (jthrowable)ex);
    (*env)->DeleteLocalRef(env, jmsg);
    (*env)->DeleteLocalRef(env, cls);
    if (ex) (*env)->DeleteLocalRef(env, ex);
}

static void throw_ctx(JNIEnv* env, omr_ctx* ctx, omr_status st) {
    throw_omr(env, st, ctx ? omr_last_error(ctx) : "");
}

static int bytes_per_pixel(jint t) {
    switch (t) {
    case OMR_PIXELS_INT8: case OMR_PIXELS_UINT8: return 1;
    case OMR_PIXELS_INT16: case OMR_PIXELS_UINT16: return 2;
    case OMR_PIXELS_INT32: case OMR_PIXELS_UINT32: case OMR_PIXELS_FLOAT: return 4;
    case OMR_PIXELS_DOUBLE: return 8;
    default: return 0;
    }
}

static jctx* get_ctx(JNIEnv* env, jlong h) {
    jctx* J = (jctx*)(intptr_t)h;
    if (!J || !J->ctx) throw_omr(env, OMR_INVALID_ARGUMENT, "null context");
    return J && J->ctx ? J : NULL;
}

/* Pinned staging of at least `bytes`.  The context keeps one grow-only buffer up to
 * STAGE_KEEP_MAX bytes (a few tiles); a larger request (a full-plane render, an 8 GiB worst-case
 * encode) gets a temporary pinned buffer that unstage() frees after the call, so one big request
 * does not stay pinned for the rest of a worker context's life. */
#define STAGE_KEEP_MAX ((size_t)64 << 20)
static uint8_t* stage(JNIEnv* env, jctx* J, size_t bytes) {
    if (bytes == 0) bytes = 1;
    if (bytes > STAGE_KEEP_MAX) {
        uint8_t* tmp = (uint8_t*)omr_pinned_alloc(J->ctx, bytes);
        if (!tmp) throw_omr(env, OMR_OOM, "pinned staging");
        return tmp;
    }
    if (bytes > J->pin_cap) {
        if (J->pin) omr_pinned_free(J->ctx, J->pin);
        J->pin_cap = 0;
        J->pin = (uint8_t*)omr_pinned_alloc(J->ctx, bytes);
        if (!J->pin) {
            throw_omr(env, OMR_OOM, "pinned staging");
            return NULL;
        }
        J->pin_cap = bytes;
    }
    return J->pin;
}

/* Release what stage() returned: a temporary buffer is freed, the kept one stays. */
static void unstage(jctx* J, uint8_t* p) {
    if (p && p != J->pin) omr_pinned_free(J->ctx, p);
}

/* 16-byte alignment of each slice of the staging buffer (planes, ARGB output, encoded bytes):
 * the library's copies and the int views stay aligned whatever the plane size. */
static size_t align16(size_t n) { return (n + 15) & ~(size_t)15; }

/* Length of a Java array that must hold at least `need` elements (INVALID_ARGUMENT otherwise). */
static int check_len(JNIEnv* env, jarray a, int64_t need, const char* what) {
    if (!a) {
        throw_omr(env, OMR_INVALID_ARGUMENT, what);
        return 0;
    }
    if (need < 0 || need > INT32_MAX || (int64_t)(*env)->GetArrayLength(env, a) < need) {
        throw_omr(env, OMR_INVALID_ARGUMENT, what);
        return 0;
    }
    return 1;
}

/* Settings packed by OmrNative.packChannel: {active, family, k, nr, reverse, start, end, gmin,
 * gmax, r, g, b, a} per channel; luts[c] a 768-byte R[256]G[256]B[256] table or null. */
typedef struct {
    omr_channel_binding cb[MAX_CH];
    uint8_t lut[MAX_CH][768];
    jsize n;
} settings;

static int load_settings(JNIEnv* env, jdoubleArray jch, jobjectArray jluts, settings* s) {
    if (!jch) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "null channel settings");
        return 0;
    }
    const jsize len = (*env)->GetArrayLength(env, jch);
    if (len <= 0 || len % NCH_FIELDS || len / NCH_FIELDS > MAX_CH) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "bad channel settings array");
        return 0;
    }
    s->n = len / NCH_FIELDS;
    if (jluts && (*env)->GetArrayLength(env, jluts) < s->n) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "LUT array shorter than the channel list");
        return 0;
    }
    jdouble d[NCH_FIELDS * MAX_CH];
    (*env)->GetDoubleArrayRegion(env, jch, 0, len, d);
    if ((*env)->ExceptionCheck(env)) return 0;
    for (jsize c = 0; c < s->n; ++c) {
        const jdouble* p = d + NCH_FIELDS * c;
        omr_channel_binding* b = &s->cb[c];
        memset(b, 0, sizeof(*b));
        b->active = (int32_t)p[0];
        b->family = (int32_t)p[1];
        b->coefficient = p[2];
        b->noise_reduction = (int32_t)p[3];
        b->reverse = (int32_t)p[4];
        b->input_start = p[5];
        b->input_end = p[6];
        b->global_min = p[7];
        b->global_max = p[8];
        for (int k = 0; k < 4; ++k) b->rgba[k] = (uint8_t)(int)p[9 + k];
        b->lut = NULL;
        if (!jluts) continue;
        jbyteArray lut = (jbyteArray)(*env)->GetObjectArrayElement(env, jluts, c);
        if ((*env)->ExceptionCheck(env)) return 0;
        if (!lut) continue;
        const int ok = (*env)->GetArrayLength(env, lut) == 768;
        if (ok) (*env)->GetByteArrayRegion(env, lut, 0, 768, (jbyte*)s->lut[c]);
        (*env)->DeleteLocalRef(env, lut);
        if (!ok) {
            throw_omr(env, OMR_INVALID_ARGUMENT, "LUT must be 768 bytes");
            return 0;
        }
        if ((*env)->ExceptionCheck(env)) return 0;
        b->lut = s->lut[c];
    }
    return 1;
}

/* ---- context ---------------------------------------------------------------------------- */
JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_create(
        JNIEnv* env, jclass cls, jint device) {
    jctx* J = (jctx*)calloc(1, sizeof(jctx));
    if (!J) {
        throw_omr(env, OMR_OOM, "context");
        return 0;
    }
    const omr_status st = omr_ctx_create(device, &J->ctx);
    if (st) {
        free(J);
        throw_omr(env, st, "omr_ctx_create failed");
        return 0;
    }
    return (jlong)(intptr_t)J;
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_destroy(
        JNIEnv* env, jclass cls, jlong h) {
    jctx* J = (jctx*)(intptr_t)h;
    if (!J) return;
    if (J->pin) omr_pinned_free(J->ctx, J->pin);
    omr_ctx_destroy(J->ctx);
    free(J);
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_setSemantics(
        JNIEnv* env, jclass cls, jlong h, jint flags) {
    jctx* J = get_ctx(env, h);
    if (!J) return;
    const omr_status st = omr_ctx_set_semantics(J->ctx, (uint32_t)flags);
    if (st) throw_ctx(env, J->ctx, st);
}

/* ---- renderAsPackedInt + flip -------------------------------------------------------------- */
JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_renderPackedInt(
        JNIEnv* env, jclass cls, jlong h, jint model, jdoubleArray jch, jobjectArray jluts,
        jobjectArray jplanes, jint pixelType, jboolean bigEndian, jint w, jint ht, jboolean flipH,
        jboolean flipV, jintArray jout) {
    jctx* J = get_ctx(env, h);
    if (!J) return;
    const int bpp = bytes_per_pixel(pixelType);
    if (!bpp || w < 0 || ht < 0) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "bad pixel type or size");
        return;
    }
    settings* s = (settings*)malloc(sizeof(settings));
    if (!s) { throw_omr(env, OMR_OOM, "settings"); return; }
    if (!load_settings(env, jch, jluts, s)) { free(s); return; }
    const int64_t npx = (int64_t)w * ht, plane_bytes = npx * bpp;
    int n_active = 0;
    for (jsize c = 0; c < s->n; ++c) n_active += s->cb[c].active ? 1 : 0;
    if (plane_bytes > INT32_MAX) {
        free(s);
        throw_omr(env, OMR_INVALID_ARGUMENT, "plane larger than a Java array");
        return;
    }
    if (!check_len(env, jplanes, s->n, "planes array shorter than the channel list") ||
        !check_len(env, jout, npx, "ARGB output shorter than width*height")) {
        free(s);
        return;
    }
    for (jsize c = 0; c < s->n; ++c) {                  /* validate every active plane first */
        if (!s->cb[c].active) continue;
        jbyteArray a = (jbyteArray)(*env)->GetObjectArrayElement(env, jplanes, c);
        if ((*env)->ExceptionCheck(env)) { free(s); return; }
        const int ok = a && (int64_t)(*env)->GetArrayLength(env, a) >= plane_bytes;
        if (a) (*env)->DeleteLocalRef(env, a);
        if (!ok) {
            free(s);
            throw_omr(env, OMR_INVALID_ARGUMENT, "active channel's plane is null or shorter than width*height");
            return;
        }
    }
    const size_t slot = align16((size_t)plane_bytes), out_off = slot * (size_t)n_active;
    uint8_t* pin = stage(env, J, out_off + (size_t)npx * 4);
    if (!pin) { free(s); return; }
    const void* planes[MAX_CH] = {0};
    size_t off = 0;
    for (jsize c = 0; c < s->n; ++c) {                  /* copy each active plane, drop its local ref */
        if (!s->cb[c].active) continue;
        jbyteArray a = (jbyteArray)(*env)->GetObjectArrayElement(env, jplanes, c);
        if ((*env)->ExceptionCheck(env)) { free(s); unstage(J, pin); return; }
        if (!a || (int64_t)(*env)->GetArrayLength(env, a) < plane_bytes) {   /* changed since the check */
            if (a) (*env)->DeleteLocalRef(env, a);
            free(s);
            unstage(J, pin);
            throw_omr(env, OMR_INVALID_ARGUMENT, "plane array changed during the call");
            return;
        }
        (*env)->GetByteArrayRegion(env, a, 0, (jsize)plane_bytes, (jbyte*)(pin + off));
        (*env)->DeleteLocalRef(env, a);
        if ((*env)->ExceptionCheck(env)) { free(s); unstage(J, pin); return; }
        planes[c] = pin + off;
        off += slot;
    }
    const omr_quantum_def q = {0, 255, 255, model};      /* createRenderingDef, :273-277 */
    const omr_status st = omr_render_packed_int(J->ctx, &q, s->cb, s->n, planes, 0, pixelType, bigEndian, w, ht,
                                                flipH, flipV, (uint32_t*)(pin + out_off));
    free(s);
    if (!st) (*env)->SetIntArrayRegion(env, jout, 0, (jsize)npx, (const jint*)(pin + out_off));
    else throw_ctx(env, J->ctx, st);
    unstage(J, pin);
}

/* ---- ProjectionService.projectStack ----------------------------------------------------------- */
JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_projectStack(
        JNIEnv* env, jclass cls, jlong h, jbyteArray jstack, jint pixelType, jboolean beIn, jint sx,
        jint sy, jint sz, jint alg, jint start, jint end, jint stepping, jbyteArray jout, jboolean beOut) {
    jctx* J = get_ctx(env, h);
    if (!J) return;
    const int bpp = bytes_per_pixel(pixelType);
    if (!bpp || sx <= 0 || sy <= 0 || sz <= 0) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "bad pixel type or stack size");
        return;
    }
    const int64_t plane = (int64_t)sx * sy * bpp, stack = plane * sz;
    if (!check_len(env, jstack, stack, "stack shorter than sizeX*sizeY*sizeZ pixels") ||
        !check_len(env, jout, plane, "plane output shorter than sizeX*sizeY pixels"))
        return;
    const size_t out_off = align16((size_t)stack);
    uint8_t* pin = stage(env, J, out_off + (size_t)plane);
    if (!pin) return;
    (*env)->GetByteArrayRegion(env, jstack, 0, (jsize)stack, (jbyte*)pin);
    if ((*env)->ExceptionCheck(env)) { unstage(J, pin); return; }
    const omr_status st = omr_project_stack(J->ctx, pin, pixelType, beIn, sx, sy, sz, alg, start, end, stepping,
                                            pin + out_off, beOut);
    if (!st) (*env)->SetByteArrayRegion(env, jout, 0, (jsize)plane, (const jbyte*)(pin + out_off));
    else throw_ctx(env, J->ctx, st);
    unstage(J, pin);
}

/* ---- encoders: ARGB int[] -> file bytes ------------------------------------------------------- */
typedef omr_status (*encode_fn)(omr_ctx*, const uint32_t*, int32_t, int32_t, uint8_t*, size_t, size_t*);

static jbyteArray new_bytes(JNIEnv* env, const uint8_t* p, size_t len) {
    if (len > INT32_MAX) {
        throw_omr(env, OMR_INTERNAL, "result larger than a Java array");
        return NULL;
    }
    jbyteArray res = (*env)->NewByteArray(env, (jsize)len);
    if (res) (*env)->SetByteArrayRegion(env, res, 0, (jsize)len, (const jbyte*)p);
    return res;
}

static jbyteArray encode(JNIEnv* env, jlong h, jintArray jargb, jint w, jint ht, int kind, float quality) {
    jctx* J = get_ctx(env, h);
    if (!J) return NULL;
    if (w <= 0 || ht <= 0) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "bad image size");
        return NULL;
    }
    const int64_t npx = (int64_t)w * ht;
    if (!check_len(env, jargb, npx, "ARGB array shorter than width*height")) return NULL;
    const size_t cap = kind == 0 ? omr_jpeg_max_bytes(w, ht) : kind == 1 ? omr_png_max_bytes(w, ht, 3)
                                                                           : omr_tiff_max_bytes(w, ht);
    const size_t buf_off = align16((size_t)npx * 4);
    uint8_t* pin = stage(env, J, buf_off + cap);
    if (!pin) return NULL;
    (*env)->GetIntArrayRegion(env, jargb, 0, (jsize)npx, (jint*)pin);
    if ((*env)->ExceptionCheck(env)) { unstage(J, pin); return NULL; }
    uint8_t* buf = pin + buf_off;
    size_t len = 0;
    const uint32_t* argb = (const uint32_t*)pin;
    const omr_status st = kind == 0 ? omr_encode_jpeg(J->ctx, argb, w, ht, quality, buf, cap, &len)
                        : kind == 1 ? omr_encode_png(J->ctx, argb, w, ht, buf, cap, &len)
                                    : omr_encode_tiff(J->ctx, argb, w, ht, buf, cap, &len);
    jbyteArray res = NULL;
    if (st) throw_ctx(env, J->ctx, st);
    else res = new_bytes(env, buf, len);
    unstage(J, pin);
    return res;
}

JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_encodeJpeg(
        JNIEnv* env, jclass cls, jlong h, jintArray jargb, jint w, jint ht, jfloat quality) {
    return encode(env, h, jargb, w, ht, 0, quality);
}

JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_encodePng(
        JNIEnv* env, jclass cls, jlong h, jintArray jargb, jint w, jint ht) {
    return encode(env, h, jargb, w, ht, 1, 0.f);
}

JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_encodeTiff(
        JNIEnv* env, jclass cls, jlong h, jintArray jargb, jint w, jint ht) {
    return encode(env, h, jargb, w, ht, 2, 0.f);
}

/* ---- ShapeMaskRequestHandler.renderShapeMask(Color, byte[], w, h) ---------------------------- */
JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_renderShapeMaskPng(
        JNIEnv* env, jclass cls, jlong h, jbyteArray jbits, jint w, jint ht, jbyteArray jrgba, jboolean flipH,
        jboolean flipV) {
    jctx* J = get_ctx(env, h);
    if (!J) return NULL;
    if (!check_len(env, jrgba, 4, "fill colour must be 4 bytes (RGBA)")) return NULL;
    uint8_t rgba[4];
    (*env)->GetByteArrayRegion(env, jrgba, 0, 4, (jbyte*)rgba);
    if ((*env)->ExceptionCheck(env)) return NULL;
    const jsize nbits = jbits ? (*env)->GetArrayLength(env, jbits) : 0;   /* null mask: the library's 404 */
    /* The library's own checks, before anything is pinned: every one of them is an exception inside
     * renderShapeMask, which ShapeMaskVerticle.java:119-128 answers with 404 (OMR_NOT_FOUND). */
    const int64_t npx = (int64_t)w * ht;
    if (w <= 0 || ht <= 0 || npx > INT32_MAX || !jbits || (int64_t)nbits * 8 < npx) {
        throw_omr(env, OMR_NOT_FOUND, w <= 0 || ht <= 0 ? "Attempted to flip image with 0 size"
                                      : npx > INT32_MAX ? "width*height overflows a Java int"
                                      : !jbits          ? "NullPointerException: null mask bytes"
                                                        : "mask shorter than width*height bits");
        return NULL;
    }
    const size_t cap = omr_png_max_bytes(w, ht, 1), buf_off = align16((size_t)nbits);
    uint8_t* pin = stage(env, J, buf_off + cap);
    if (!pin) return NULL;
    (*env)->GetByteArrayRegion(env, jbits, 0, nbits, (jbyte*)pin);
    if ((*env)->ExceptionCheck(env)) { unstage(J, pin); return NULL; }
    size_t len = 0;
    uint8_t* buf = pin + buf_off;
    const omr_status st = omr_render_shape_mask_png(J->ctx, pin, (size_t)nbits, w, ht, rgba, flipH, flipV, buf, cap,
                                                    &len);
    jbyteArray res = NULL;
    if (st) throw_ctx(env, J->ctx, st);
    else res = new_bytes(env, buf, len);
    unstage(J, pin);
    return res;
}

/* ---- ROMIO pixel buffer + request batcher + node pool ----------------------------------------- */
JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_pixelBufferOpen(
        JNIEnv* env, jclass cls, jstring jpath, jint sx, jint sy, jint sz, jint sc, jint st_, jint pixelType) {
    if (!jpath) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "null path");
        return 0;
    }
    const char* path = (*env)->GetStringUTFChars(env, jpath, NULL);
    if (!path) return 0;                                 /* OutOfMemoryError pending */
    omr_pixel_buffer* pb = NULL;
    const omr_status st = omr_pixel_buffer_open(path, sx, sy, sz, sc, st_, pixelType, &pb);
    (*env)->ReleaseStringUTFChars(env, jpath, path);
    if (st) throw_omr(env, st, "omr_pixel_buffer_open failed");
    return (jlong)(intptr_t)pb;
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_pixelBufferClose(
        JNIEnv* env, jclass cls, jlong pb) {
    omr_pixel_buffer_close((omr_pixel_buffer*)(intptr_t)pb);
}

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_batcherCreate(
        JNIEnv* env, jclass cls, jint device, jint maxBatch, jint maxWaitUs) {
    omr_batcher* b = NULL;
    const omr_status st = omr_batcher_create(device, maxBatch, maxWaitUs, &b);
    if (st) throw_omr(env, st, "omr_batcher_create failed");
    return (jlong)(intptr_t)b;
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_batcherDestroy(
        JNIEnv* env, jclass cls, jlong b) {
    omr_batcher_destroy((omr_batcher*)(intptr_t)b);
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_batcherSetSemantics(
        JNIEnv* env, jclass cls, jlong b, jint flags) {
    const omr_status st = omr_batcher_set_semantics((omr_batcher*)(intptr_t)b, (uint32_t)flags);
    if (st) throw_omr(env, st, "unknown semantics flag");
}

typedef omr_status (*submit_fn)(void*, const omr_tile_job*, uint64_t*);
typedef omr_status (*wait_fn)(void*, uint64_t, uint8_t*, size_t, size_t*);

static jlong submit(JNIEnv* env, void* q, submit_fn fn, jlong jpb, jint model, jdoubleArray jch, jobjectArray jluts,
                    jint z, jint t, jint x, jint y, jint w, jint h, jboolean flipH, jboolean flipV, jint format,
                    jfloat quality) {
    if (!q || !jpb) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "null batcher or pixel buffer");
        return 0;
    }
    settings* s = (settings*)malloc(sizeof(settings));
    if (!s) { throw_omr(env, OMR_OOM, "settings"); return 0; }
    if (!load_settings(env, jch, jluts, s)) { free(s); return 0; }
    const omr_quantum_def qd = {0, 255, 255, model};
    omr_tile_job job;
    memset(&job, 0, sizeof(job));                        /* no projection */
    job.pb = (const omr_pixel_buffer*)(intptr_t)jpb;
    job.qdef = &qd;
    job.channels = s->cb;
    job.size_c = s->n;
    job.z = z;
    job.t = t;
    job.x = x;
    job.y = y;
    job.width = w;
    job.height = h;
    job.flip_h = flipH;
    job.flip_v = flipV;
    job.format = format;
    job.quality = quality;
    uint64_t ticket = 0;
    const omr_status st = fn(q, &job, &ticket);          /* copies the settings and LUTs */
    free(s);
    if (st) throw_omr(env, st, st == OMR_NOT_FOUND ? "unknown format" : "submit failed");
    return (jlong)ticket;
}

static jbyteArray wait_result(JNIEnv* env, void* q, wait_fn fn, jlong ticket) {
    if (!q) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "null batcher");
        return NULL;
    }
    size_t len = 0;
    omr_status st = fn(q, (uint64_t)ticket, NULL, 0, &len);        /* size query; the result is kept */
    if (st != OMR_BUFFER_TOO_SMALL && st != OMR_OK) {
        throw_omr(env, st, "tile request failed");
        return NULL;
    }
    uint8_t* buf = (uint8_t*)malloc(len ? len : 1);
    if (!buf) { throw_omr(env, OMR_OOM, "result buffer"); return NULL; }
    st = fn(q, (uint64_t)ticket, buf, len, &len);
    jbyteArray res = NULL;
    if (st) throw_omr(env, st, "tile request failed");
    else res = new_bytes(env, buf, len);
    free(buf);
    return res;
}

/* p=intmax|intmean|intsum at t (ImageRegionRequestHandler.java:506-558): the full plane; start / end
 * < 0 take the reference's defaults (0 / sizeZ - 1). */
static jlong submit_projected(JNIEnv* env, void* q, submit_fn fn, jlong jpb, jint model, jdoubleArray jch,
                              jobjectArray jluts, jint t, jint alg, jint start, jint end, jboolean flipH,
                              jboolean flipV, jint format, jfloat quality) {
    if (!q || !jpb) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "null batcher or pixel buffer");
        return 0;
    }
    settings* s = (settings*)malloc(sizeof(settings));
    if (!s) { throw_omr(env, OMR_OOM, "settings"); return 0; }
    if (!load_settings(env, jch, jluts, s)) { free(s); return 0; }
    const omr_quantum_def qd = {0, 255, 255, model};
    omr_tile_job job;
    memset(&job, 0, sizeof(job));
    job.pb = (const omr_pixel_buffer*)(intptr_t)jpb;
    job.qdef = &qd;
    job.channels = s->cb;
    job.size_c = s->n;
    job.t = t;
    job.flip_h = flipH;
    job.flip_v = flipV;
    job.format = format;
    job.quality = quality;
    job.has_projection = 1;
    job.projection = alg;
    job.projection_start = start;
    job.projection_end = end;
    uint64_t ticket = 0;
    const omr_status st = fn(q, &job, &ticket);
    free(s);
    if (st) throw_omr(env, st, st == OMR_NOT_FOUND ? "unknown format" : "submit failed");
    return (jlong)ticket;
}

typedef omr_status (*submit_mask_fn)(void*, const omr_mask_job*, uint64_t*);

/* render_shape_mask (ShapeMaskRequestHandler.java:165-207) as a queued job: the mask bytes are
 * copied by the library at submit; every 404 case of the reference fails the job at wait. */
static jlong submit_mask(JNIEnv* env, void* q, submit_mask_fn fn, jbyteArray jbits, jint w, jint ht,
                         jbyteArray jrgba, jboolean flipH, jboolean flipV) {
    if (!q) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "null batcher");
        return 0;
    }
    if (!check_len(env, jrgba, 4, "fill colour must be 4 bytes (RGBA)")) return 0;
    omr_mask_job job;
    memset(&job, 0, sizeof(job));
    (*env)->GetByteArrayRegion(env, jrgba, 0, 4, (jbyte*)job.rgba);
    if ((*env)->ExceptionCheck(env)) return 0;
    const jsize nbits = jbits ? (*env)->GetArrayLength(env, jbits) : 0;
    uint8_t* bits = NULL;
    if (jbits) {                                         /* null stays null: the job's 404 */
        bits = (uint8_t*)malloc(nbits ? (size_t)nbits : 1);
        if (!bits) { throw_omr(env, OMR_OOM, "mask copy"); return 0; }
        if (nbits) (*env)->GetByteArrayRegion(env, jbits, 0, nbits, (jbyte*)bits);
        if ((*env)->ExceptionCheck(env)) { free(bits); return 0; }
    }
    job.bits = bits;
    job.n_bytes = (size_t)nbits;
    job.width = w;
    job.height = ht;
    job.flip_h = flipH;
    job.flip_v = flipV;
    uint64_t ticket = 0;
    const omr_status st = fn(q, &job, &ticket);          /* copies the mask */
    free(bits);
    if (st) throw_omr(env, st, "submit failed");
    return (jlong)ticket;
}

static omr_status batcher_submit_mask(void* q, const omr_mask_job* j, uint64_t* t) {
    return omr_batcher_submit_mask((omr_batcher*)q, j, t);
}
static omr_status pool_submit_mask(void* q, const omr_mask_job* j, uint64_t* t) {
    return omr_pool_submit_mask((omr_pool*)q, j, t);
}

static omr_status batcher_submit(void* q, const omr_tile_job* j, uint64_t* t) {
    return omr_batcher_submit((omr_batcher*)q, j, t);
}
static omr_status batcher_wait(void* q, uint64_t t, uint8_t* o, size_t c, size_t* n) {
    return omr_batcher_wait((omr_batcher*)q, t, o, c, n);
}
static omr_status pool_submit(void* q, const omr_tile_job* j, uint64_t* t) {
    return omr_pool_submit((omr_pool*)q, j, t);
}
static omr_status pool_wait(void* q, uint64_t t, uint8_t* o, size_t c, size_t* n) {
    return omr_pool_wait((omr_pool*)q, t, o, c, n);
}

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_batcherSubmit(
        JNIEnv* env, jclass cls, jlong jb, jlong jpb, jint model, jdoubleArray jch, jobjectArray jluts, jint z,
        jint t, jint x, jint y, jint w, jint h, jboolean flipH, jboolean flipV, jint format, jfloat quality) {
    return submit(env, (void*)(intptr_t)jb, batcher_submit, jpb, model, jch, jluts, z, t, x, y, w, h, flipH, flipV,
                  format, quality);
}

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_batcherSubmitProjected(
        JNIEnv* env, jclass cls, jlong jb, jlong jpb, jint model, jdoubleArray jch, jobjectArray jluts, jint t,
        jint alg, jint start, jint end, jboolean flipH, jboolean flipV, jint format, jfloat quality) {
    return submit_projected(env, (void*)(intptr_t)jb, batcher_submit, jpb, model, jch, jluts, t, alg, start, end,
                            flipH, flipV, format, quality);
}

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_batcherSubmitMask(
        JNIEnv* env, jclass cls, jlong jb, jbyteArray jbits, jint w, jint ht, jbyteArray jrgba, jboolean flipH,
        jboolean flipV) {
    return submit_mask(env, (void*)(intptr_t)jb, batcher_submit_mask, jbits, w, ht, jrgba, flipH, flipV);
}

JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_batcherWait(
        JNIEnv* env, jclass cls, jlong jb, jlong ticket) {
    return wait_result(env, (void*)(intptr_t)jb, batcher_wait, ticket);
}

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_poolCreate(
        JNIEnv* env, jclass cls, jintArray jdevices, jint maxBatch, jint maxWaitUs) {
    if (!check_len(env, jdevices, 1, "device list must not be empty")) return 0;
    const jsize n = (*env)->GetArrayLength(env, jdevices);
    if (n > 256) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "at most 256 devices");
        return 0;
    }
    jint dev[256];
    (*env)->GetIntArrayRegion(env, jdevices, 0, n, dev);
    if ((*env)->ExceptionCheck(env)) return 0;
    int32_t d32[256];
    for (jsize i = 0; i < n; ++i) d32[i] = dev[i];
    omr_pool* p = NULL;
    const omr_status st = omr_pool_create(d32, n, maxBatch, maxWaitUs, &p);
    if (st) throw_omr(env, st, "omr_pool_create failed");
    return (jlong)(intptr_t)p;
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_poolDestroy(
        JNIEnv* env, jclass cls, jlong p) {
    omr_pool_destroy((omr_pool*)(intptr_t)p);
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_poolSetSemantics(
        JNIEnv* env, jclass cls, jlong p, jint flags) {
    const omr_status st = omr_pool_set_semantics((omr_pool*)(intptr_t)p, (uint32_t)flags);
    if (st) throw_omr(env, st, "unknown semantics flag");
}

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_poolSubmit(
        JNIEnv* env, jclass cls, jlong jp, jlong jpb, jint model, jdoubleArray jch, jobjectArray jluts, jint z,
        jint t, jint x, jint y, jint w, jint h, jboolean flipH, jboolean flipV, jint format, jfloat quality) {
    return submit(env, (void*)(intptr_t)jp, pool_submit, jpb, model, jch, jluts, z, t, x, y, w, h, flipH, flipV,
                  format, quality);
}

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_poolSubmitProjected(
        JNIEnv* env, jclass cls, jlong jp, jlong jpb, jint model, jdoubleArray jch, jobjectArray jluts, jint t,
        jint alg, jint start, jint end, jboolean flipH, jboolean flipV, jint format, jfloat quality) {
    return submit_projected(env, (void*)(intptr_t)jp, pool_submit, jpb, model, jch, jluts, t, alg, start, end,
                            flipH, flipV, format, quality);
}

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_poolSubmitMask(
        JNIEnv* env, jclass cls, jlong jp, jbyteArray jbits, jint w, jint ht, jbyteArray jrgba, jboolean flipH,
        jboolean flipV) {
    return submit_mask(env, (void*)(intptr_t)jp, pool_submit_mask, jbits, w, ht, jrgba, flipH, flipV);
}

JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_poolWait(
        JNIEnv* env, jclass cls, jlong jp, jlong ticket) {
    return wait_result(env, (void*)(intptr_t)jp, pool_wait, ticket);
}
