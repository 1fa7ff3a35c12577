"""Time render variants in one process (kernel-only, HIP events) to split the frame
cost into primary / shadow / shading phases.  Usage: python tools/ablate.py [iters]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
ctx = DeviceContext(0)
rows = []
import os
only = os.environ.get("ABLATE_SCENES")
modes = os.environ.get("ABLATE_MODES")
for name, W, H in [("W4_Bunny", 1920, 1080), ("W3", 1280, 720), ("W4_Reference", 1920, 1080),
                   ("W4_Optional", 1920, 1080), ("Synthetic100k", 1920, 1080), ("Bunny8Lights", 3840, 2160),
                   ("W1", 640, 480)]:
    if only and name not in only.split(","):
        continue
    hs = HostScene(name)
    s, cam = hs.view()
    ctx.upload(s)
    for mode, sh, tag in [(3, 1, "combined+shadows"), (3, 0, "combined"), (0, 0, "observed-area"),
                          (1, 0, "radiance")]:
        if modes and tag not in modes.split(","):
            continue
        p = abi.make_params(W, H, mode, sh)
        ctx.time_frames(cam, p, 5)
        # ABLATE_WARM=<ms>: render continuously that long first, so the GPU clock has left its
        # idle state (profiles/r02/warmup_probe.txt) — light variants otherwise run slow clocks
        import time
        t_end = time.perf_counter() + float(os.environ.get("ABLATE_WARM", "0")) / 1e3
        while time.perf_counter() < t_end:
            ctx.time_frames(cam, p, 50)
        ms = min(ctx.time_frames(cam, p, iters) for _ in range(3))
        flop = None
        if tag == "combined+shadows":
            import numpy as np
            c = ctx.count_work(cam, p)
            cost = [41, 19, 14, 12, 63, 9, 15, 1, 26, 6, 31, 103]
            flop = int(sum(int(a) * b for a, b in zip(c, cost)))
        mpix = W * H / ms / 1e3
        line = f"{name:14s} {W}x{H} {tag:18s} {ms*1e3:9.1f} us  {mpix:9.1f} Mpix/s"
        if flop:
            line += f"  {flop / (ms * 1e-3) / 1e12:6.2f} TFLOP/s ({flop / (W * H):.0f} FLOP/px)"
        print(line, flush=True)
