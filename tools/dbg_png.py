import sys, os, zlib, struct
sys.path.insert(0, "/root/repo/omero-ms-image-region_amd"); sys.path.insert(0, "/root/repo/tests")
import numpy as np, torch
import omr, oracle_lib as O
from omr import _lib
from omr.synthetic import c2_channels, tile_u16
planes = tile_u16(3, 4, 512, 512)
st, argb = O.render(c2_channels(4), planes, _lib.PIXELS_UINT16, 512, 512)
def idat(png):
    i, out = 8, b""
    while i < len(png):
        ln, = struct.unpack(">I", png[i:i+4])
        if png[i+4:i+8] == b"IDAT": out += png[i+8:i+8+ln]
        i += 12 + ln
    return out
with omr.Context(0) as ctx:
    a = ctx.encode_png(argb, 512, 512)
    b = ctx.encode_png(argb, 512, 512)
    d = torch.from_numpy(argb.view(np.int32)).to("cuda")
    c = ctx.encode_png_device(d, 512, 512)
    for name, x in (("host2", b), ("dev", c)):
        ia, ix = idat(a), idat(x)
        print(name, len(ia), len(ix), a == x)
        if ia != ix:
            k = next(i for i in range(min(len(ia), len(ix))) if ia[i] != ix[i]) if ia[:min(len(ia),len(ix))] != ix[:min(len(ia),len(ix))] else min(len(ia),len(ix))
            print(" first diff at", k)
            da, dx = zlib.decompress(ia), zlib.decompress(ix)
            print(" decompressed equal:", da == dx, len(da), len(dx))
            if da != dx:
                k2 = next(i for i in range(len(da)) if da[i] != dx[i]); print(" raw diff at", k2, "row", k2 // 1537)
