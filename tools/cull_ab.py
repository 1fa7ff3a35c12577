"""A/B of the exact cull on one GPU: every BASELINE config (and the other mesh
scenes) rendered by contexts created under different cull settings (environment variables read
by rtx_create: RTX_NO_CULL, RTX_CULL_*, and the split / tile-order knobs RTX_SPLIT*, RTX_TILE_ORDER).
CULL_AB_SCENES=a,b restricts the configs.  Checks every setting's frame is
bit-identical to the unculled one (uint32 and float planes) and prints kernel ms/frame of each
(rtx_time_frames: HIP events, mean over `iters` serialized launches, best of 3).

Usage (GPU box): python tools/cull_ab.py [iters] [out.json] [setting ...]
  setting = name=VAR:value,VAR:value  (default: the product default and RTX_NO_CULL=1)
"""
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

CONFIGS = [("W4_Bunny", 1920, 1080), ("W4_Optional", 1920, 1080), ("Synthetic100k", 1920, 1080),
           ("Bunny8Lights", 3840, 2160), ("W4_Reference", 1920, 1080), ("W3", 1280, 720), ("W1", 640, 480)]
KNOBS = ("RTX_NO_CULL", "RTX_CULL_RATIO", "RTX_CULL_LEAVES", "RTX_CULL_MIN_SA", "RTX_SPLIT", "RTX_SPLIT_FACTOR",
         "RTX_SPLIT_PARTS", "RTX_TILE_ORDER")


def ctx_with(env: dict) -> DeviceContext:
    saved = {k: os.environ.pop(k, None) for k in KNOBS}
    os.environ.update(env)
    try:
        return DeviceContext(0)
    finally:
        for k in KNOBS:
            os.environ.pop(k, None)
            if saved[k] is not None:
                os.environ[k] = saved[k]


def parse(arg: str):
    name, _, rest = arg.partition("=")
    env = dict(kv.split(":", 1) for kv in rest.split(",") if kv)
    return name, env


def main() -> None:
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    out = Path(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] != "-" else None
    settings = [parse(a) for a in sys.argv[3:]] or [("cull", {})]
    settings = [("no_cull", {"RTX_NO_CULL": "1"})] + settings
    rows = []
    only = os.environ.get("CULL_AB_SCENES")
    for name, W, H in CONFIGS:
        if only and name not in only.split(","):
            continue
        hs = HostScene(name)
        s, cam = hs.view()
        p = abi.make_params(W, H)
        res = {"config": f"{name} {W}x{H}"}
        base = None
        for tag, env in settings:
            ctx = ctx_with(env)
            ctx.upload(s)
            for _ in range(4):   # cost-ordered and split state live, as bench.py times it
                px, rgb = ctx.render(cam, p)
            res[f"{tag}_ms"] = round(min(ctx.time_frames(cam, p, iters) for _ in range(3)), 5)
            ctx.close()
            if base is None:
                base = (px, rgb)
            else:
                same = bool(np.array_equal(px, base[0]) and np.array_equal(rgb.view(np.uint32), base[1].view(np.uint32)))
                res[f"{tag}_bit_identical"] = same
                res[f"{tag}_speedup"] = round(res["no_cull_ms"] / res[f"{tag}_ms"], 4)
        print(json.dumps(res), flush=True)
        rows.append(res)
    if out:
        out.write_text(json.dumps(rows, indent=1) + "\n")
    if not all(v for r in rows for k, v in r.items() if k.endswith("_bit_identical")):
        sys.exit(1)


if __name__ == "__main__":
    main()
