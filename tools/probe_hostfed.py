"""Host-fed bandwidth probe: pread (tmpfs -> pageable / pinned) and PCIe H2D / D2H rates."""
import os, sys, time, tempfile
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "omero-ms-image-region_amd"))
import numpy as np
import torch
from concurrent.futures import ThreadPoolExecutor
from omr import PixelBuffer, _lib, write_romio

X = Y = 4096
img = np.random.default_rng(0).integers(0, 65536, (1, 4, 1, Y, X), dtype=np.uint16)
fd, path = tempfile.mkstemp(dir="/dev/shm"); os.close(fd)
write_romio(path, img, _lib.PIXELS_UINT16)
pb = PixelBuffer(path, X, Y, 1, 4, 1, _lib.PIXELS_UINT16)
out = np.empty((1024, 1024), dtype=">u2")
t0 = time.perf_counter()
for i in range(64):
    _lib.lib.omr_pixel_buffer_get_tile(pb.h, 0, i % 4, 0, (i // 4 % 4) * 1024, 0, 1024, 1024, out.ctypes.data, out.nbytes)
el = time.perf_counter() - t0
print(f"pread 1 thread, 1024-px rows: {64 * 2 / el / 1024:.2f} GB/s")
band = np.empty((1024, 4096), dtype=">u2")
t0 = time.perf_counter()
for i in range(16):
    _lib.lib.omr_pixel_buffer_get_tile(pb.h, 0, i % 4, 0, 0, (i // 4) * 1024, 4096, 1024, band.ctypes.data, band.nbytes)
el = time.perf_counter() - t0
print(f"pread 1 thread, full-width band: {16 * 8 / el / 1024:.2f} GB/s")
for nt in (4, 8, 16):
    bufs = [np.empty((1024, 1024), dtype=">u2") for _ in range(nt)]
    def job(i):
        b = bufs[i % nt]
        _lib.lib.omr_pixel_buffer_get_tile(pb.h, 0, i % 4, 0, (i // 4 % 4) * 1024, (i // 16 % 4) * 1024, 1024, 1024, b.ctypes.data, b.nbytes)
    with ThreadPoolExecutor(nt) as ex:
        list(ex.map(job, range(nt)))
        t0 = time.perf_counter()
        list(ex.map(job, range(256)))
        el = time.perf_counter() - t0
    print(f"pread {nt} threads: {256 * 2 / el / 1024:.2f} GB/s")
print("os.cpu_count", os.cpu_count(), "sched_getaffinity", len(os.sched_getaffinity(0)))
h = torch.empty(64 << 20, dtype=torch.uint8).pin_memory()
d = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
for name, fn in [("H2D pinned", lambda: d.copy_(h, non_blocking=True)), ("D2H pinned", lambda: h.copy_(d, non_blocking=True))]:
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"{name}: {10 * 64 / el / 1024:.2f} GB/s")
os.unlink(path)
