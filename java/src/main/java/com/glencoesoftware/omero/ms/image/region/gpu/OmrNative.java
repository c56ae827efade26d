package com.glencoesoftware.omero.ms.image.region.gpu;

/**
 * JNI facade over libomr.so (jni/omr_jni.c, include/omr/omr.h).  One context per Vert.x worker
 * thread (contexts are not thread-safe; distinct contexts may run concurrently), or one shared
 * batcher per GPU, or one pool over the node's GPUs for every worker.  Every native method throws
 * {@link OmrException} on failure; array arguments are copied in and out (no critical region is
 * held across a GPU call), and a short or null array is INVALID_ARGUMENT.
 *
 * Paths are relative to src/main/java/com/glencoesoftware/omero/ms/image/region/ of the reference.
 * Not compiled in this repository's image (no JDK); the C side it binds is built and tested here.
 */
public final class OmrNative implements AutoCloseable {
    static {
        System.loadLibrary("omr_jni");   // libomr_jni.so, linked against libomr.so
    }

    /** include/omr/omr.h enums. */
    public static final int PIXELS_INT8 = 0, PIXELS_UINT8 = 1, PIXELS_INT16 = 2, PIXELS_UINT16 = 3,
            PIXELS_INT32 = 4, PIXELS_UINT32 = 5, PIXELS_FLOAT = 6, PIXELS_DOUBLE = 7;
    public static final int FAMILY_LINEAR = 0, FAMILY_POLYNOMIAL = 1, FAMILY_LOGARITHMIC = 2,
            FAMILY_EXPONENTIAL = 3;
    public static final int MODEL_GREYSCALE = 0, MODEL_RGB = 1;
    public static final int FORMAT_JPEG = 0, FORMAT_PNG = 1, FORMAT_ARGB = 2, FORMAT_TIFF = 3;
    public static final int PROJECTION_MAX = 0, PROJECTION_MEAN = 1, PROJECTION_SUM = 2;
    /** OMR_SEM_* switches of the un-vendored upstream semantics. */
    public static final int SEM_WINDOW_INT_BOUNDS = 1, SEM_ALPHA_SEPARATE = 2, SEM_GREYSCALE_LUT = 4,
            SEM_JPEG_CHROMA_DIV2 = 8, SEM_PROJECTION_ALL_ACTIVE = 16, SEM_LOG_UNGUARDED = 32,
            SEM_NOISE_REDUCTION_OFF = 64, SEM_EXP_NORMALIZED = 128, SEM_MASK_PIXEL_FLIP = 256;
    /** doubles per channel in the packed settings array. */
    public static final int CHANNEL_FIELDS = 13;

    private final long ctx;

    public OmrNative(int device) {
        ctx = create(device);
    }

    public long handle() {
        return ctx;
    }

    @Override
    public void close() {
        destroy(ctx);
    }

    /**
     * One ChannelBinding after createRenderingDef + updateSettings
     * (ImageRegionRequestHandler.java:281-298, :689-741) into settings[c*13 .. c*13+12].
     */
    public static void packChannel(double[] settings, int c, boolean active, int family, double coefficient,
                                   boolean noiseReduction, boolean reverse, double windowStart,
                                   double windowEnd, double globalMin, double globalMax, int[] rgba) {
        final int o = c * CHANNEL_FIELDS;
        settings[o] = active ? 1 : 0;
        settings[o + 1] = family;
        settings[o + 2] = coefficient;
        settings[o + 3] = noiseReduction ? 1 : 0;
        settings[o + 4] = reverse ? 1 : 0;
        settings[o + 5] = windowStart;
        settings[o + 6] = windowEnd;
        settings[o + 7] = globalMin;
        settings[o + 8] = globalMax;
        for (int k = 0; k < 4; k++) {
            settings[o + 9 + k] = rgba[k];
        }
    }

    // ---- context ------------------------------------------------------------------------
    private static native long create(int device);
    private static native void destroy(long ctx);
    public static native void setSemantics(long ctx, int flags);

    // ---- renderer.renderAsPackedInt + flip (:559, :574-575) -------------------------------
    /** planes[c]: the region of channel c as raw bytes (ROMIO: big-endian), null if inactive. */
    public static native void renderPackedInt(long ctx, int model, double[] settings, byte[][] luts,
                                              byte[][] planes, int pixelType, boolean bigEndian,
                                              int width, int height, boolean flipH, boolean flipV,
                                              int[] argbOut);

    // ---- ProjectionService.projectStack (ProjectionService.java:46-120) ----------------------
    public static native void projectStack(long ctx, byte[] stack, int pixelType, boolean bigEndianIn,
                                           int sizeX, int sizeY, int sizeZ, int algorithm, int start,
                                           int end, int stepping, byte[] planeOut, boolean bigEndianOut);

    // ---- encoders (:576-600) --------------------------------------------------------------------
    /** compressToStream with the quality passed per call (no shared setCompressionLevel). */
    public static native byte[] encodeJpeg(long ctx, int[] argb, int width, int height, float quality);
    public static native byte[] encodePng(long ctx, int[] argb, int width, int height);
    public static native byte[] encodeTiff(long ctx, int[] argb, int width, int height);

    // ---- ShapeMaskRequestHandler.renderShapeMask(Color, byte[], w, h) (:165-207) -----------------
    public static native byte[] renderShapeMaskPng(long ctx, byte[] bits, int width, int height, byte[] rgba,
                                                   boolean flipH, boolean flipV);

    // ---- ROMIO pixel buffer (getPixelBuffer, :302-309) + batcher (one per GPU) --------------------
    public static native long pixelBufferOpen(String path, int sizeX, int sizeY, int sizeZ, int sizeC,
                                              int sizeT, int pixelType);
    public static native void pixelBufferClose(long pixelBuffer);
    public static native long batcherCreate(int device, int maxBatch, int maxWaitUs);
    public static native void batcherDestroy(long batcher);
    /** Returns a ticket; the job's settings are copied, the pixel buffer must outlive the job. */
    public static native long batcherSubmit(long batcher, long pixelBuffer, int model, double[] settings,
                                            byte[][] luts, int z, int t, int x, int y, int width, int height,
                                            boolean flipH, boolean flipV, int format, float quality);
    /**
     * A p=intmax|intmean|intsum request (ImageRegionRequestHandler.java:506-558): every active channel
     * projected (PROJECTION_*) over z in [start, end] at t (negative: 0 / sizeZ - 1), the full plane
     * rendered and encoded.
     */
    public static native long batcherSubmitProjected(long batcher, long pixelBuffer, int model, double[] settings,
                                                     byte[][] luts, int t, int algorithm, int start, int end,
                                                     boolean flipH, boolean flipV, int format, float quality);
    /** render_shape_mask (ShapeMaskRequestHandler.java:165-207); wait returns the PNG (404 cases throw). */
    public static native long batcherSubmitMask(long batcher, byte[] bits, int width, int height, byte[] rgba,
                                                boolean flipH, boolean flipV);
    /** Blocks until the job is done; the encoded tile (JPEG / PNG / TIFF) or the packed ARGB bytes. */
    public static native byte[] batcherWait(long batcher, long ticket);
    /** OMR_SEM_* flags for jobs submitted after this call. */
    public static native void batcherSetSemantics(long batcher, int flags);

    // ---- node pool: one batcher per GPU (ImageRegionMicroserviceVerticle.java:84-85, :149-165) -------
    /** devices[i]: the GPU ordinal of batcher i (may repeat); jobs go to the least-queued batcher. */
    public static native long poolCreate(int[] devices, int maxBatch, int maxWaitUs);
    public static native void poolDestroy(long pool);
    public static native void poolSetSemantics(long pool, int flags);
    public static native long poolSubmit(long pool, long pixelBuffer, int model, double[] settings,
                                         byte[][] luts, int z, int t, int x, int y, int width, int height,
                                         boolean flipH, boolean flipV, int format, float quality);
    public static native long poolSubmitProjected(long pool, long pixelBuffer, int model, double[] settings,
                                                  byte[][] luts, int t, int algorithm, int start, int end,
                                                  boolean flipH, boolean flipV, int format, float quality);
    public static native long poolSubmitMask(long pool, byte[] bits, int width, int height, byte[] rgba,
                                             boolean flipH, boolean flipV);
    public static native byte[] poolWait(long pool, long ticket);
}
