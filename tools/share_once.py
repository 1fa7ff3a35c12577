"""Render rank 0's share of a frame cut into 16-row stripes over s ranks, `frames` times on one
context (serialized), for kernel traces (rocprofv3 --kernel-trace --stats -- python tools/share_once.py ...).
Usage: python tools/share_once.py <scene> <W> <H> <s> [frames]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

scene, W, H, st = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
frames = int(sys.argv[5]) if len(sys.argv) > 5 else 50
hs = HostScene(scene)
s, cam = hs.view()
ctx = DeviceContext(0)
ctx.upload(s)
p = abi.make_params(W, H, stripe_rows=16 if st > 1 else 0, stripe_first=0, stripe_step=st)
ms = C.c_float()
# ~1000 untimed frames first: a fresh process starts the GPU at its idle clock (Measurement)
abi.check(ctx.lib.rtx_time_views(ctx.h, cam, 1, C.byref(p), int(1000 * 0.05 / max(0.01, 0.4 / st)), C.byref(ms)), "w",
          ctx.h)
abi.check(ctx.lib.rtx_time_views(ctx.h, cam, 1, C.byref(p), frames, C.byref(ms)), "t", ctx.h)
print(f"{scene} {W}x{H} s={st}: {ms.value:.5f} ms per frame (serialized), light-major {ctx.light_major_info()[0]}, "
      f"heavy {ctx.split_info()[0]}, parts {ctx.split_info()[1]}")
ctx.close()
