"""Frames in flight: K frames of one view rendered through 1, 2 or 3 render contexts on
the same GPU (each its own stream, buffers and schedule), issued round robin, so that a
frame's tail overlaps the next frame's start.  Prints the per-frame wall time.
Usage: python tools/pipeline_probe.py [scene W H steps]"""
import ctypes as C
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "W4_Bunny"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
H = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
K = int(sys.argv[4]) if len(sys.argv) > 4 else 400
hs = HostScene(name)
s, cam = hs.view()
p = abi.make_params(W, H)
ctxs = [DeviceContext(0) for _ in range(3)]
for c in ctxs:
    c.upload(s)
for n in (1, 2, 3, 1, 2, 3):
    use = ctxs[:n]
    for i in range(60):
        c = use[i % n]
        abi.check(c.lib.rtx_render_async(c.h, C.byref(cam), C.byref(p), 0), "render", c.h)
    for c in use:
        c.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        c = use[i % n]
        abi.check(c.lib.rtx_render_async(c.h, C.byref(cam), C.byref(p), 0), "render", c.h)
    for c in use:
        c.synchronize()
    dt = (time.perf_counter() - t0) / K
    print(f"{name} {W}x{H}: {n} context(s) in flight: {dt * 1e6:7.1f} us/frame  {W * H / dt / 1e6:9.1f} Mpix/s",
          flush=True)
