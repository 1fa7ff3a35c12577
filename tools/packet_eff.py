"""Packet efficiency of the wave traversal: lane-level slab/triangle tests (the
reference's per-ray work) vs what the waves executed (64 lanes x node-pair / triangle
steps).  Usage: python tools/packet_eff.py"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

ctx = DeviceContext(0)
for name, W, H in [("W4_Bunny", 1920, 1080), ("W4_Optional", 1920, 1080), ("Synthetic100k", 1920, 1080),
                   ("Bunny8Lights", 3840, 2160)]:
    hs = HostScene(name)
    s, cam = hs.view()
    ctx.upload(s)
    for sh in (0, 1):
        p = abi.make_params(W, H, 3, sh)
        out = (C.c_uint64 * 14)()
        abi.check(ctx.lib.rtx_count_work_ex(ctx.h, C.byref(cam), C.byref(p), out, 14), "count", ctx.h)
        c = list(out)
        npx = W * H
        slab_lane, tri_lane, node_w, tri_w = c[3], c[4], c[12], c[13]
        print(f"{name:14s} shadows={sh}: per px  slab {slab_lane/npx:7.2f} tri {tri_lane/npx:7.2f} | "
              f"wave slab-eff {slab_lane/max(1, (2*node_w+1)*64):.3f} tri-eff {tri_lane/max(1, tri_w*64):.3f} | "
              f"per wave: node-pair steps {node_w/(npx/64):8.1f} tri steps {tri_w/(npx/64):8.1f}", flush=True)
