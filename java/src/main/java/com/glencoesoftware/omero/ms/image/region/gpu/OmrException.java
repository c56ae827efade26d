package com.glencoesoftware.omero.ms.image.region.gpu;

/**
 * A libomr.so call failed.  {@link #status} is the omr_status code (include/omr/omr.h);
 * {@link #httpStatus()} is the outcome the reference answers with for the same failure
 * (ImageRegionVerticle.java:163-186, ImageRegionMicroserviceVerticle.java:301-304).
 */
public final class OmrException extends RuntimeException {
    public static final int INVALID_ARGUMENT = 1, NOT_FOUND = 2, QUANTIZATION = 3, DEVICE = 4, OOM = 5,
            BUFFER_TOO_SMALL = 6, INTERNAL = 7;

    public final int status;

    public OmrException(int status, String message) {
        super("omr status " + status + ": " + message);
        this.status = status;
    }

    public int httpStatus() {
        switch (status) {
            case INVALID_ARGUMENT: return 400;
            case NOT_FOUND: return 404;
            default: return 500;
        }
    }
}
