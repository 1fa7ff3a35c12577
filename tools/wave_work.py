"""Per-wave packet work of the instrumented kernel: node-pair and triangle steps per wave
(rtx_count_work_ex diagnostics) next to the per-pixel model counts.
Usage: python tools/wave_work.py [scene W H ...]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

NAMES = ["pixels", "sphere", "plane", "slab", "tri", "hit", "shadow", "occluded", "shade", "lambert", "phong", "ct",
         "wave_node_pairs", "wave_tri_steps"]
args = sys.argv[1:] or ["W4_Bunny", "1920", "1080", "W3", "1280", "720", "W4_Optional", "1920", "1080"]
ctx = DeviceContext(0)
for i in range(0, len(args), 3):
    name, W, H = args[i], int(args[i + 1]), int(args[i + 2])
    hs = HostScene(name)
    s, cam = hs.view()
    ctx.upload(s)
    p = abi.make_params(W, H, 3, 1)
    out = (C.c_uint64 * 14)()
    abi.check(ctx.lib.rtx_count_work_ex(ctx.h, C.byref(cam), C.byref(p), out, 14), "rtx_count_work_ex", ctx.h)
    c = list(out)
    waves = ((W + 7) // 8) * ((H + 7) // 8)
    px = c[0]
    per_px = " ".join(f"{n} {c[k] / px:.2f}" for k, n in enumerate(NAMES[1:12], 1))
    print(f"{name} {W}x{H}: waves {waves}  per wave: node pairs {c[12] / waves:.2f}  tri steps {c[13] / waves:.2f}"
          f"  | per px: {per_px}", flush=True)
