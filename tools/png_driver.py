"""Drive the PNG encoders for profiling: a rendered C2 tile and a 1024^2 shape mask."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "omero-ms-image-region_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
import torch
import omr
import oracle_lib as O
from omr import _lib
from omr.synthetic import c2_channels, tile_u16
planes = tile_u16(3, 4, 1024, 1024)
st, argb = O.render(c2_channels(4), planes, _lib.PIXELS_UINT16, 1024, 1024)
yy, xx = np.mgrid[0:1024, 0:1024]
m = ((yy - 500) / 300.0) ** 2 + ((xx - 400) / 200.0) ** 2 <= 1
bits = np.packbits(m.reshape(-1)).tobytes()
with omr.Context(0) as ctx:
    d = torch.from_numpy(argb.view(np.int32)).to("cuda")
    for i in range(10):
        ctx.encode_png_device(d, 1024, 1024)
        ctx.render_shape_mask_png(bits, 1024, 1024, (255, 0, 0, 128), True, True)
print("ok")
