"""omr — MI355X-native image-region rendering (Python side of the drop-in).

Layers:
  _lib      ctypes binding of libomr.so (the C ABI in include/omr/omr.h)
  context   Context: one per worker thread / GPU (device, stream, workspace)
  renderer  Renderer facade mirroring the omeis Renderer calls the reference makes
            (ImageRegionRequestHandler.java:436-440, :689-741, :559)
  pixbuf    PixelBuffer: ROMIO repository pixel files (getPixelBuffer, :302-309)
  batcher   Batcher: concurrent requests coalesced into GPU batches; Pool: one batcher per GPU
  request   ImageRegionCtx / ShapeMaskCtx parsing and the handler glue
            (ImageRegionCtx.java, ImageRegionRequestHandler.java, ShapeMaskRequestHandler.java)
"""
from . import _lib
from ._lib import OmrError
from .context import Context
from .pixbuf import PixelBuffer, write_romio
from .batcher import Batcher, Pool
from .renderer import (ChannelSettings, Renderer, ReverseIntensityContext, create_rendering_def,
                       flip, split_html_color)
from .request import (ImageRegionCtx, ImageRegionRequestHandler, InMemoryPixelBuffer, LutProvider,
                      RequestError, ShapeMaskCtx, ShapeMaskRequestHandler)

__all__ = ["_lib", "OmrError", "Context", "Renderer", "ChannelSettings", "ReverseIntensityContext",
           "create_rendering_def", "flip", "split_html_color", "ImageRegionCtx",
           "ImageRegionRequestHandler", "InMemoryPixelBuffer", "LutProvider", "RequestError",
           "ShapeMaskCtx", "ShapeMaskRequestHandler", "PixelBuffer", "write_romio", "Batcher", "Pool"]
