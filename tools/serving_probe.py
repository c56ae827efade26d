#!/usr/bin/env python3
"""Batcher serving from a ROMIO file, for same-box A/B of the dispatcher count
(OMR_BATCH_LANES in this process's environment): 8 client threads, 8 JPEG tiles (1024^2, C2
settings, q 0.9) in flight each, 256 requests per pass; (a) the bench's pattern (16 distinct tiles
of t 0, most requests deduplicated), (b) 64 distinct tiles over 4 timepoints.  Second of two passes
timed.  One JSON line: answered and rendered tiles/s, p50 latency."""
import json
import os
import sys
import tempfile
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "omero-ms-image-region_amd"))


def main():
    import numpy as np
    import omr
    from omr import Batcher, PixelBuffer, _lib, write_romio
    from omr.context import make_bindings, make_qdef
    from omr.synthetic import c2_channels
    T, grid, C, NT = 1024, 4, 4, 4
    rng = np.random.default_rng(5)
    img = rng.integers(0, 65536, (NT, C, 1, grid * T, grid * T), dtype=np.uint16)
    fd, path = tempfile.mkstemp(prefix="omr_serve_", dir="/dev/shm")
    os.close(fd)
    res = {"workers": os.environ.get("OMR_BATCH_LANES", "default")}
    try:
        write_romio(path, img, _lib.PIXELS_UINT16)
        del img
        qd, chans = make_qdef("rgb"), c2_channels(C)
        binds = make_bindings(chans)
        pb = PixelBuffer(path, grid * T, grid * T, 1, C, NT, _lib.PIXELS_UINT16)
        n_req, clients = 256, 8
        pats = {"16_distinct": [(0, 0, (i % grid) * T, ((i // grid) % grid) * T) for i in range(n_req)],
                "64_distinct": [(0, (i // 16) % NT, (i % grid) * T, ((i // grid) % grid) * T) for i in range(n_req)]}
        with Batcher(0, max_batch=64, max_wait_us=1000) as b:
            for name, reqs in pats.items():
                lats = []

                def client(k):
                    mine = list(range(k, n_req, clients))
                    for s0 in range(0, len(mine), 8):
                        a = time.perf_counter()
                        ts = [b.submit(pb, qd, chans, *reqs[i], T, T, quality=0.9, bindings=binds) for i in mine[s0:s0 + 8]]
                        for t in ts:
                            b.wait(t)
                            lats.append(time.perf_counter() - a)
                s0 = b.stats()
                for warm in (True, False):
                    lats.clear()
                    if not warm:
                        s0 = b.stats()
                    ths = [threading.Thread(target=client, args=(k,)) for k in range(clients)]
                    t0 = time.perf_counter()
                    for t in ths:
                        t.start()
                    for t in ths:
                        t.join()
                    el = time.perf_counter() - t0
                s1 = b.stats()
                rendered = s1["rendered"] - s0["rendered"]
                res[name] = {"tiles_per_s": round(n_req / el, 1), "rendered_per_s": round(rendered / el, 1),
                             "p50_ms": round(1e3 * float(np.median(lats)), 3),
                             "rounds": s1["batches"] - s0["batches"]}
        pb.close()
    finally:
        os.unlink(path)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
