"""MI355X-native drop-in for the per-pixel render loop of GP1_Raytracer_2223.

Layers:
  include/rtx.h          C-ABI render boundary  -> lib/librtx_hip.so  (HIP, gfx950)
  include/rtx_host.h     C++ host scene layer   -> lib/librtx_host.so (g++)
  renderer.Renderer      Python mirror of dae::Renderer over the C-ABI
"""
from . import abi  # noqa: F401

__all__ = ["abi"]
