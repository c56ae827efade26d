#!/usr/bin/env python3
"""Generate the committed golden vectors in tests/golden/.

jpeg_golden.npz — the external pin of the JPEG path.  Inputs are small seeded RGB images
(ragged sizes exercise IJG edge replication and dummy blocks); outputs are encoded by
PIL 12.2 / libjpeg-turbo 3.1 (islow FDCT, 4:2:0, standard Huffman tables) using the
quantisation tables Java ImageIO derives from the request quality
(JPEG.convertToLinearQuality + JPEGQTable.getScaledInstance, the JDK writer behind
compressionService.compressToStream, ImageRegionRequestHandler.java:581).  libjpeg-turbo is
the IJG 6b lineage the JDK bundles; its islow/quantise/Huffman stages are bit-compatible.

render_golden.npz — regression fixtures of the CPU restatement (oracle/liboracle.so) on the
C2 settings; they pin the oracle against drift, they do not pin it against Java (that
arithmetic is un-vendored: see oracle/omr_oracle.c, "UNPINNED").

Run from the repo root:  python tests/golden/make_golden.py
"""
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "omero-ms-image-region_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

JPEG_CASES = [  # (width, height, quality, pattern)
    (64, 64, 0.9, "gradient"), (64, 64, 0.9, "noise"), (37, 53, 0.85, "noise"),
    (37, 53, 0.85, "gradient"), (1, 1, 0.5, "noise"), (17, 9, 0.3, "gradient"),
    (16, 17, 1.0, "noise"), (130, 66, 0.05, "noise"), (48, 32, 0.8, "flat"),
]


def java_quant_tables(q):
    """javax.imageio: linear = q<0.5 ? 0.5/q : 2-2q (float); entry (int)(std*linear + 0.5f)."""
    std_l = [16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
             14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
             49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99]
    std_c = [17, 18, 24, 47] + [99] * 4 + [18, 21, 26, 66] + [99] * 4 + [24, 26, 56] + [99] * 5 + [47, 66] + [99] * 38
    f = np.float32
    qf = f(q)
    if qf <= f(0):
        qf = f(0.01)
    if qf > f(1):
        qf = f(1)
    qf = f(0.5) / qf if qf < f(0.5) else f(2) - qf * f(2)
    mk = lambda t: [int(min(255, max(1, int(f(v) * qf + f(0.5))))) for v in t]
    return mk(std_l), mk(std_c)


def pattern(w, h, kind, seed):
    rng = np.random.default_rng(seed)
    if kind == "noise":
        return rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    if kind == "flat":
        return np.full((h, w, 3), (12, 200, 77), np.uint8)
    yy, xx = np.mgrid[0:h, 0:w]
    return np.stack([(xx * 3) % 256, (yy * 5) % 256, ((xx + yy) * 2) % 256], -1).astype(np.uint8)


def main():
    from PIL import Image, features
    out = {}
    for i, (w, h, q, kind) in enumerate(JPEG_CASES):
        rgb = pattern(w, h, kind, 1000 + i)
        ql, qc = java_quant_tables(q)
        buf = io.BytesIO()
        Image.fromarray(rgb, "RGB").save(buf, "JPEG", qtables=[ql, qc], subsampling=2)
        out[f"rgb_{i}"] = rgb
        out[f"jpeg_{i}"] = np.frombuffer(buf.getvalue(), np.uint8)
        out[f"meta_{i}"] = np.array([w, h, q], np.float64)
        out[f"qtab_{i}"] = np.array(ql + qc, np.uint8)
    out["libjpeg_turbo"] = np.array(str(features.version("libjpeg_turbo")))
    np.savez_compressed(os.path.join(HERE, "jpeg_golden.npz"), **out)

    import oracle_lib as O
    from omr import _lib
    from omr.synthetic import c2_channels, tile_u16
    planes = tile_u16(77, 4, 48, 64)
    be = [p.astype(">u2") for p in planes]
    st, argb = O.render(c2_channels(4), be, _lib.PIXELS_UINT16, 64, 48, big_endian=True)
    assert st == 0
    st2, argb_flip = O.render(c2_channels(4), be, _lib.PIXELS_UINT16, 64, 48, big_endian=True, flip_h=True, flip_v=True)
    np.savez_compressed(os.path.join(HERE, "render_golden.npz"), planes=np.stack(planes), argb=argb,
                        argb_flip_hv=argb_flip)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
