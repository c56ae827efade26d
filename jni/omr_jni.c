/*
 * omr_jni.c — JNI shim between the reference's Java host code and libomr.so (include/omr/omr.h).
 *
 * Java side: java/src/main/java/com/glencoesoftware/omero/ms/image/region/gpu/OmrNative.java.
 * Build (needs a JDK, absent from this image — see jni/Makefile and INTEGRATION.md §3):
 *   make -C jni JAVA_HOME=/usr/lib/jvm/java-8-openjdk-amd64
 *
 * Call sites it serves (paths relative to src/main/java/com/glencoesoftware/omero/ms/image/region/):
 *   renderPackedInt     renderer.renderAsPackedInt + flip      ImageRegionRequestHandler.java:559, :574-575
 *   projectStack        projectionService.projectStack         ProjectionService.java:46-120
 *   encodeJpeg          compressionService.compressToStream     ImageRegionRequestHandler.java:576-582
 *   encodePng/Tiff      ImageIO.write / TIFFImageWriter         ImageRegionRequestHandler.java:583-600
 *   renderShapeMaskPng  renderShapeMask(Color, byte[], w, h)    ShapeMaskRequestHandler.java:165-207
 *   batcher*            one Renderer per request on each worker ImageRegionMicroserviceVerticle.java:149-165
 *
 * Rules kept here: no JNI call while a critical array is held (object references and LUT bytes
 * are fetched first); every acquired array is released on every path; library failures become
 * OmrException(status, message) whose status maps to the reference's HTTP outcome (omr.h).
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "omr/omr.h"

#define PKG "com/glencoesoftware/omero/ms/image/region/gpu/"
#define NCH_FIELDS 13          /* doubles per channel in the packed settings array (OmrNative.java) */
#define MAX_CH OMR_MAX_REQUEST_CHANNELS

static void throw_omr(JNIEnv* env, jint status, const char* msg) {
    jclass cls = (*env)->FindClass(env, PKG "OmrException");
    if (!cls) return;                                   /* NoClassDefFoundError already pending */
    jmethodID ctor = (*env)->GetMethodID(env, cls, "<init>", "(ILjava/lang/String;)V");
    jstring jmsg = (*env)->NewStringUTF(env, msg ? msg : "");
    jobject ex = (*env)->NewObject(env, cls, ctor, status, jmsg);
    if (ex) (*env)->Throw(env, (jthrowable)ex);
}

static void throw_ctx(JNIEnv* env, omr_ctx* ctx, omr_status st) {
    throw_omr(env, st, ctx ? omr_last_error(ctx) : "");
}

/* Settings packed by OmrNative.packChannel: {active, family, k, nr, reverse, start, end, gmin,
 * gmax, r, g, b, a} per channel; luts[c] a 768-byte R[256]G[256]B[256] table or null. */
typedef struct {
    omr_channel_binding cb[MAX_CH];
    uint8_t lut[MAX_CH][768];
    jsize n;
} settings;

static int load_settings(JNIEnv* env, jdoubleArray jch, jobjectArray jluts, settings* s) {
    const jsize len = (*env)->GetArrayLength(env, jch);
    if (len % NCH_FIELDS || len / NCH_FIELDS > MAX_CH) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "bad channel settings array");
        return 0;
    }
    s->n = len / NCH_FIELDS;
    jdouble d[NCH_FIELDS * MAX_CH];
    (*env)->GetDoubleArrayRegion(env, jch, 0, len, d);
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
        jbyteArray lut = jluts ? (jbyteArray)(*env)->GetObjectArrayElement(env, jluts, c) : NULL;
        if (lut) {
            if ((*env)->GetArrayLength(env, lut) != 768) {
                throw_omr(env, OMR_INVALID_ARGUMENT, "LUT must be 768 bytes");
                return 0;
            }
            (*env)->GetByteArrayRegion(env, lut, 0, 768, (jbyte*)s->lut[c]);
            b->lut = s->lut[c];
            (*env)->DeleteLocalRef(env, lut);
        }
    }
    return 1;
}

/* ---- context ---------------------------------------------------------------------------- */
JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_create(
        JNIEnv* env, jclass cls, jint device) {
    omr_ctx* ctx = NULL;
    const omr_status st = omr_ctx_create(device, &ctx);
    if (st) throw_omr(env, st, "omr_ctx_create failed");
    return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_destroy(
        JNIEnv* env, jclass cls, jlong ctx) {
    omr_ctx_destroy((omr_ctx*)(intptr_t)ctx);
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_setSemantics(
        JNIEnv* env, jclass cls, jlong jctx, jint flags) {
    omr_ctx* ctx = (omr_ctx*)(intptr_t)jctx;
    const omr_status st = omr_ctx_set_semantics(ctx, (uint32_t)flags);
    if (st) throw_ctx(env, ctx, st);
}

/* ---- renderAsPackedInt + flip -------------------------------------------------------------- */
JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_renderPackedInt(
        JNIEnv* env, jclass cls, jlong jctx, jint model, jdoubleArray jch, jobjectArray jluts,
        jobjectArray jplanes, jint pixelType, jboolean bigEndian, jint w, jint h, jboolean flipH,
        jboolean flipV, jintArray jout) {
    omr_ctx* ctx = (omr_ctx*)(intptr_t)jctx;
    settings* s = (settings*)malloc(sizeof(settings));
    if (!s) { throw_omr(env, OMR_OOM, "settings"); return; }
    if (!load_settings(env, jch, jluts, s)) { free(s); return; }
    if ((*env)->GetArrayLength(env, jplanes) < s->n || (*env)->GetArrayLength(env, jout) < (jsize)w * h) {
        free(s);
        throw_omr(env, OMR_INVALID_ARGUMENT, "planes / output too short");
        return;
    }
    jbyteArray arrs[MAX_CH];
    const void* planes[MAX_CH];
    for (jsize c = 0; c < s->n; ++c)                     /* all JNI calls before the critical section */
        arrs[c] = (jbyteArray)(*env)->GetObjectArrayElement(env, jplanes, c);
    for (jsize c = 0; c < s->n; ++c)
        planes[c] = arrs[c] ? (*env)->GetPrimitiveArrayCritical(env, arrs[c], NULL) : NULL;
    jint* out = (jint*)(*env)->GetPrimitiveArrayCritical(env, jout, NULL);
    const omr_quantum_def q = {0, 255, 255, model};      /* createRenderingDef, :273-277 */
    const omr_status st = omr_render_packed_int(ctx, &q, s->cb, s->n, planes, 0, pixelType, bigEndian, w, h,
                                                flipH, flipV, (uint32_t*)out);
    (*env)->ReleasePrimitiveArrayCritical(env, jout, out, st ? JNI_ABORT : 0);
    for (jsize c = s->n - 1; c >= 0; --c)
        if (arrs[c]) (*env)->ReleasePrimitiveArrayCritical(env, arrs[c], (void*)planes[c], JNI_ABORT);
    free(s);
    if (st) throw_ctx(env, ctx, st);
}

/* ---- ProjectionService.projectStack ----------------------------------------------------------- */
JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_projectStack(
        JNIEnv* env, jclass cls, jlong jctx, jbyteArray jstack, jint pixelType, jboolean beIn, jint sx,
        jint sy, jint sz, jint alg, jint start, jint end, jint stepping, jbyteArray jout, jboolean beOut) {
    omr_ctx* ctx = (omr_ctx*)(intptr_t)jctx;
    void* stack = (*env)->GetPrimitiveArrayCritical(env, jstack, NULL);
    void* out = (*env)->GetPrimitiveArrayCritical(env, jout, NULL);
    const omr_status st = omr_project_stack(ctx, stack, pixelType, beIn, sx, sy, sz, alg, start, end, stepping,
                                            out, beOut);
    (*env)->ReleasePrimitiveArrayCritical(env, jout, out, st ? JNI_ABORT : 0);
    (*env)->ReleasePrimitiveArrayCritical(env, jstack, stack, JNI_ABORT);
    if (st) throw_ctx(env, ctx, st);
}

/* ---- encoders: ARGB int[] -> file bytes ------------------------------------------------------- */
typedef omr_status (*encode_fn)(omr_ctx*, const uint32_t*, int32_t, int32_t, uint8_t*, size_t, size_t*);

static jbyteArray encode(JNIEnv* env, omr_ctx* ctx, jintArray jargb, jint w, jint h, size_t cap, encode_fn fn,
                         int jpeg, float quality) {
    if ((*env)->GetArrayLength(env, jargb) < (jsize)w * h) {
        throw_omr(env, OMR_INVALID_ARGUMENT, "ARGB array too short");
        return NULL;
    }
    uint8_t* buf = (uint8_t*)malloc(cap);
    if (!buf) { throw_omr(env, OMR_OOM, "encode buffer"); return NULL; }
    size_t len = 0;
    jint* argb = (jint*)(*env)->GetPrimitiveArrayCritical(env, jargb, NULL);
    const omr_status st = jpeg ? omr_encode_jpeg(ctx, (const uint32_t*)argb, w, h, quality, buf, cap, &len)
                               : fn(ctx, (const uint32_t*)argb, w, h, buf, cap, &len);
    (*env)->ReleasePrimitiveArrayCritical(env, jargb, argb, JNI_ABORT);
    jbyteArray res = NULL;
    if (st) {
        throw_ctx(env, ctx, st);
    } else if ((res = (*env)->NewByteArray(env, (jsize)len)) != NULL) {
        (*env)->SetByteArrayRegion(env, res, 0, (jsize)len, (const jbyte*)buf);
    }
    free(buf);
    return res;
}

JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_encodeJpeg(
        JNIEnv* env, jclass cls, jlong jctx, jintArray jargb, jint w, jint h, jfloat quality) {
    return encode(env, (omr_ctx*)(intptr_t)jctx, jargb, w, h, omr_jpeg_max_bytes(w, h), NULL, 1, quality);
}

JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_encodePng(
        JNIEnv* env, jclass cls, jlong jctx, jintArray jargb, jint w, jint h) {
    return encode(env, (omr_ctx*)(intptr_t)jctx, jargb, w, h, omr_png_max_bytes(w, h, 3), omr_encode_png, 0, 0.f);
}

JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_encodeTiff(
        JNIEnv* env, jclass cls, jlong jctx, jintArray jargb, jint w, jint h) {
    return encode(env, (omr_ctx*)(intptr_t)jctx, jargb, w, h, omr_tiff_max_bytes(w, h), omr_encode_tiff, 0, 0.f);
}

/* ---- ShapeMaskRequestHandler.renderShapeMask(Color, byte[], w, h) ---------------------------- */
JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_renderShapeMaskPng(
        JNIEnv* env, jclass cls, jlong jctx, jbyteArray jbits, jint w, jint h, jbyteArray jrgba, jboolean flipH,
        jboolean flipV) {
    omr_ctx* ctx = (omr_ctx*)(intptr_t)jctx;
    uint8_t rgba[4];
    (*env)->GetByteArrayRegion(env, jrgba, 0, 4, (jbyte*)rgba);
    const jsize nbits = (*env)->GetArrayLength(env, jbits);
    const size_t cap = omr_png_max_bytes(w, h, 1);
    uint8_t* buf = (uint8_t*)malloc(cap);
    if (!buf) { throw_omr(env, OMR_OOM, "encode buffer"); return NULL; }
    size_t len = 0;
    void* bits = (*env)->GetPrimitiveArrayCritical(env, jbits, NULL);
    const omr_status st = omr_render_shape_mask_png(ctx, (const uint8_t*)bits, (size_t)nbits, w, h, rgba, flipH,
                                                    flipV, buf, cap, &len);
    (*env)->ReleasePrimitiveArrayCritical(env, jbits, bits, JNI_ABORT);
    jbyteArray res = NULL;
    if (st) throw_ctx(env, ctx, st);
    else if ((res = (*env)->NewByteArray(env, (jsize)len)) != NULL)
        (*env)->SetByteArrayRegion(env, res, 0, (jsize)len, (const jbyte*)buf);
    free(buf);
    return res;
}

/* ---- ROMIO pixel buffer + request batcher ----------------------------------------------------- */
JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_pixelBufferOpen(
        JNIEnv* env, jclass cls, jstring jpath, jint sx, jint sy, jint sz, jint sc, jint st_, jint pixelType) {
    const char* path = (*env)->GetStringUTFChars(env, jpath, NULL);
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

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_batcherSubmit(
        JNIEnv* env, jclass cls, jlong jb, jlong jpb, jint model, jdoubleArray jch, jobjectArray jluts, jint z,
        jint t, jint x, jint y, jint w, jint h, jboolean flipH, jboolean flipV, jint format, jfloat quality) {
    settings* s = (settings*)malloc(sizeof(settings));
    if (!s) { throw_omr(env, OMR_OOM, "settings"); return 0; }
    if (!load_settings(env, jch, jluts, s)) { free(s); return 0; }
    const omr_quantum_def q = {0, 255, 255, model};
    omr_tile_job job = {(const omr_pixel_buffer*)(intptr_t)jpb, &q, s->cb, s->n, z, t, x, y, w, h, flipH, flipV,
                        format, quality};
    uint64_t ticket = 0;
    const omr_status st = omr_batcher_submit((omr_batcher*)(intptr_t)jb, &job, &ticket);   /* copies settings */
    free(s);
    if (st) throw_omr(env, st, st == OMR_NOT_FOUND ? "unknown format" : "omr_batcher_submit failed");
    return (jlong)ticket;
}

JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_image_region_gpu_OmrNative_batcherWait(
        JNIEnv* env, jclass cls, jlong jb, jlong ticket) {
    omr_batcher* b = (omr_batcher*)(intptr_t)jb;
    size_t len = 0;
    omr_status st = omr_batcher_wait(b, (uint64_t)ticket, NULL, 0, &len);      /* size query; result kept */
    if (st != OMR_BUFFER_TOO_SMALL && st != OMR_OK) {
        throw_omr(env, st, "tile request failed");
        return NULL;
    }
    uint8_t* buf = (uint8_t*)malloc(len ? len : 1);
    if (!buf) { throw_omr(env, OMR_OOM, "result buffer"); return NULL; }
    st = omr_batcher_wait(b, (uint64_t)ticket, buf, len, &len);
    jbyteArray res = NULL;
    if (st) throw_omr(env, st, "tile request failed");
    else if ((res = (*env)->NewByteArray(env, (jsize)len)) != NULL)
        (*env)->SetByteArrayRegion(env, res, 0, (jsize)len, (const jbyte*)buf);
    free(buf);
    return res;
}
