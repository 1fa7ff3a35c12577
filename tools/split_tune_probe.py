"""The split threshold's tuner on one GPU: per scene, a fresh context renders frames
(serialized, rtx_time_frames) and the tuner's state is printed as it converges; then the tuned
frame time beside fixed factors (RTX_SPLIT_FACTOR: tuner off).  Every frame of every setting is
checked bit for bit against the first setting's.
Usage (GPU box): python tools/split_tune_probe.py [scene,...] [factor,...]"""
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402


def ctx_with(factor):
    saved = os.environ.pop("RTX_SPLIT_FACTOR", None)
    if factor:
        os.environ["RTX_SPLIT_FACTOR"] = factor
    try:
        return DeviceContext(0)
    finally:
        os.environ.pop("RTX_SPLIT_FACTOR", None)
        if saved is not None:
            os.environ["RTX_SPLIT_FACTOR"] = saved


def main() -> int:
    scenes = sys.argv[1].split(",") if len(sys.argv) > 1 else ["Synthetic100k", "W4_Optional", "Bunny8Lights"]
    factors = sys.argv[2].split(",") if len(sys.argv) > 2 else ["1.5", "2"]
    for name in scenes:
        W, H = (3840, 2160) if name == "Bunny8Lights" else (1920, 1080)
        hs = HostScene(name)
        s, cam = hs.view()
        p = abi.make_params(W, H)
        row = {"config": f"{name} {W}x{H}"}
        base = None
        for tag in ["tuned"] + factors:
            ctx = ctx_with(None if tag == "tuned" else tag)
            ctx.upload(s)
            trace = []
            for k in range(24):   # 4 frames per step: the tuner's progress
                ctx.time_frames(cam, p, 4)
                if tag == "tuned":
                    t = ctx.split_tune_info()
                    trace.append((4 * (k + 1), t["factor"], round(t["main_ms"], 3), round(t["chain_ms"], 3), t["state"]))
            ms = min(ctx.time_frames(cam, p, 30) for _ in range(3))
            px, rgb = ctx.render(cam, p)
            row[f"{tag}_ms"] = round(ms, 5)
            row[f"{tag}_heavy"] = ctx.split_info()[0]
            if tag == "tuned":
                row["tuner"] = ctx.split_tune_info()
                row["trace"] = trace
            if base is None:
                base = (px, rgb)
            else:
                row[f"{tag}_bit_identical"] = bool(np.array_equal(px, base[0]) and
                                                   np.array_equal(rgb.view(np.uint32), base[1].view(np.uint32)))
            ctx.close()
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
