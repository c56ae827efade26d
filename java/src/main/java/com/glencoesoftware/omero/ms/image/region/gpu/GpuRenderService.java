package com.glencoesoftware.omero.ms.image.region.gpu;

import java.io.IOException;
import java.util.Map;

import com.glencoesoftware.omero.ms.image.region.ImageRegionCtx;

/**
 * The body of ImageRegionRequestHandler.render (:496-604) on the GPU.  The handler keeps
 * everything before it (canRead, caches, metadata, getRegionDef / checkPlaneDef) and replaces
 *
 *   projection loop + renderer.renderAsPackedInt + flip + createBufferedImage + encode
 *
 * with {@link #render}.  Settings come from the request exactly as updateSettings (:689-741)
 * applies them to a fresh createRenderingDef (:258-300): linear family, k = 1, no noise
 * reduction, Float windows widened to double, HTML colour or .lut table, reverse-intensity maps.
 *
 * Not compiled in this repository's image (no JDK); OmrNative's C side is built and tested here.
 */
public final class GpuRenderService {

    /** Raw planes of the request (the reference reads them through its PixelBuffer). */
    public interface PlaneSource {
        /** Region [x, x+w) x [y, y+h) of plane (z, c, t), file byte order (ROMIO: big-endian). */
        byte[] region(int z, int c, int t, int x, int y, int w, int h) throws IOException;
        /** Whole stack of channel c at t: sizeZ planes back to back (ProjectionService.java:72). */
        byte[] stack(int c, int t) throws IOException;
    }

    /** .lut tables by name (LutProviderImpl.java:63-73); null when no such table exists. */
    public interface LutSource {
        byte[] table768(String name);
    }

    private final OmrNative gpu;

    public GpuRenderService(OmrNative gpu) {
        this.gpu = gpu;
    }

    /**
     * updateSettings (:689-741) over createRenderingDef defaults (:281-298): channel c uses the
     * request's c-th window / colour / map entry when active; inactive channels keep the
     * defaults (type range, red).  The colour parser is the reference's own public
     * ImageRegionRequestHandler.splitHTMLColor (:865-890).
     */
    static double[] settings(ImageRegionCtx ctx, int sizeC, double typeMin, double typeMax, byte[][] lutsOut,
                             LutSource luts) {
        double[] s = new double[sizeC * OmrNative.CHANNEL_FIELDS];
        for (int c = 0; c < sizeC; c++) {
            final boolean active = ctx.channels.contains(c + 1);
            double start = typeMin, end = typeMax;
            int[] rgba = {255, 0, 0, 255};
            boolean reverse = false;
            if (active) {
                if (ctx.windows != null) {
                    start = ctx.windows.get(c)[0];
                    end = ctx.windows.get(c)[1];
                }
                if (ctx.colors != null) {
                    String color = ctx.colors.get(c);
                    if (color.endsWith(".lut")) {
                        lutsOut[c] = luts != null ? luts.table768(color) : null;
                    } else {
                        rgba = com.glencoesoftware.omero.ms.image.region.ImageRegionRequestHandler
                                .splitHTMLColor(color);
                    }
                }
                if (ctx.maps != null && c < ctx.maps.size() && ctx.maps.get(c) != null) {
                    Map<String, Object> rev = ctx.maps.get(c).get("reverse");
                    reverse = rev != null && Boolean.TRUE.equals(rev.get("enabled"));
                }
            }
            OmrNative.packChannel(s, c, active, OmrNative.FAMILY_LINEAR, 1.0, false, reverse, start, end,
                                  typeMin, typeMax, rgba);
        }
        return s;
    }

    /**
     * render (:496-604) for a region of sizeX x sizeY at (x, y), or the projected full plane.
     * Returns the encoded bytes, or null for an unknown format (-> 404, :602-603).
     */
    public byte[] render(ImageRegionCtx ctx, PlaneSource src, LutSource luts, int pixelType, boolean bigEndian,
                         int sizeC, int sizeZ, int planeSizeX, int planeSizeY, int x, int y, int sizeX, int sizeY,
                         double typeMin, double typeMax) throws IOException {
        byte[][] lutTables = new byte[sizeC][];
        double[] settings = settings(ctx, sizeC, typeMin, typeMax, lutTables, luts);
        // :735-740 (a null m is an NPE -> 500 in the reference)
        int model = ctx.m.equals("greyscale") ? OmrNative.MODEL_GREYSCALE : OmrNative.MODEL_RGB;
        byte[][] planes = new byte[sizeC][];
        int w = sizeX, h = sizeY;
        if (ctx.projection != null) {
            // projection glue (:506-558): full plane; the kernel side reproduces the sizeC quirk
            // (Appendix B 3) unless OmrNative.SEM_PROJECTION_ALL_ACTIVE is set on the context
            int start = ctx.projectionStart != null ? ctx.projectionStart : 0;
            int end = ctx.projectionEnd != null ? ctx.projectionEnd : sizeZ - 1;
            w = planeSizeX;
            h = planeSizeY;
            int active = 0;
            for (int c = 0; c < sizeC; c++) {
                if (settings[c * OmrNative.CHANNEL_FIELDS] != 0) {
                    active++;
                }
            }
            int bpp = bytesPerPixel(pixelType);
            for (int c = 0; c < sizeC; c++) {
                if (settings[c * OmrNative.CHANNEL_FIELDS] == 0) {
                    continue;
                }
                if (c >= active) {   // InMemoryPlanarPixelBuffer bounds check (quirk 3)
                    throw new OmrException(OmrException.INTERNAL, "C '" + c + "' greater than sizeC '" + active + "'");
                }
                planes[c] = new byte[w * h * bpp];
                OmrNative.projectStack(gpu.handle(), src.stack(c, ctx.t), pixelType, bigEndian, w, h, sizeZ,
                                       ctx.projection, start, end, 1, planes[c], bigEndian);
            }
        } else {
            for (int c = 0; c < sizeC; c++) {
                if (settings[c * OmrNative.CHANNEL_FIELDS] != 0) {
                    planes[c] = src.region(ctx.z, c, ctx.t, x, y, w, h);
                }
            }
        }
        int[] argb = new int[w * h];
        OmrNative.renderPackedInt(gpu.handle(), model, settings, lutTables, planes, pixelType, bigEndian, w, h,
                                  ctx.flipHorizontal, ctx.flipVertical, argb);   // flip folded in (:574-575)
        switch (ctx.format) {
            case "jpeg":
                float q = ctx.compressionQuality != null ? ctx.compressionQuality : 0.85f;
                return OmrNative.encodeJpeg(gpu.handle(), argb, w, h, q);             // :580-582
            case "png":
                return OmrNative.encodePng(gpu.handle(), argb, w, h);                 // :597-599
            case "tif":
                return OmrNative.encodeTiff(gpu.handle(), argb, w, h);                // :583-596
            default:
                return null;                                                          // :602-603
        }
    }

    static int bytesPerPixel(int pixelType) {
        switch (pixelType) {
            case OmrNative.PIXELS_INT8: case OmrNative.PIXELS_UINT8: return 1;
            case OmrNative.PIXELS_INT16: case OmrNative.PIXELS_UINT16: return 2;
            case OmrNative.PIXELS_DOUBLE: return 8;
            default: return 4;
        }
    }
}
