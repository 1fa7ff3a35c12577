"""Strong-scaling diagnosis on one GPU: rank 0's share of a frame cut into 16-row stripes over s
ranks, timed alone (rtx_time_views), with the heavy-tile count the schedule splits, under context
settings given as environment variables read by rtx_create (e.g. RTX_SPLIT=0, RTX_TILE_ORDER=0).

Usage (GPU box): [SHARE_ROWS=16] [SHARE_ALL_RANKS=1] python tools/share_probe.py <scene> <W> <H> [setting ...]
  setting = name=VAR:value,VAR:value   (default: the product settings)
"""
import ctypes as C
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

KNOBS = ("RTX_SPLIT", "RTX_TILE_ORDER", "RTX_SPLIT_FACTOR", "RTX_SPLIT_PARTS", "RTX_NO_CULL")


def ctx_with(env):
    saved = {k: os.environ.pop(k, None) for k in KNOBS}
    os.environ.update(env)
    try:
        return DeviceContext(0)
    finally:
        for k in KNOBS:
            os.environ.pop(k, None)
            if saved[k] is not None:
                os.environ[k] = saved[k]


def main():
    scene, W, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    settings = [("default", {})]
    for a in sys.argv[4:]:
        n, _, rest = a.partition("=")
        settings.append((n, dict(kv.split(":", 1) for kv in rest.split(",") if kv)))
    hs = HostScene(scene)
    s, cam = hs.view()
    for name, env in settings:
        ctx = ctx_with(env)
        ctx.upload(s)
        row = {"setting": name}
        rows = int(os.environ.get("SHARE_ROWS", "16"))   # stripe height
        ranks = os.environ.get("SHARE_ALL_RANKS") == "1"   # time every rank's share (else rank 0's)
        for st in (1, 2, 4, 8):
            times = []
            for first in (range(st) if ranks else [0]):
                p = abi.make_params(W, H, stripe_rows=rows if st > 1 else 0, stripe_first=first, stripe_step=st)
                ms = C.c_float()
                abi.check(ctx.lib.rtx_time_views(ctx.h, cam, 1, C.byref(p), 5, C.byref(ms)), "t", ctx.h)
                best = 1e9
                for _ in range(2):
                    abi.check(ctx.lib.rtx_time_views(ctx.h, cam, 1, C.byref(p), 30, C.byref(ms)), "t", ctx.h)
                    best = min(best, ms.value)
                times.append(best)
            heavy, parts = ctx.split_info()
            row[f"s{st}"] = {"ms": round(max(times), 4), "rank0_ms": round(times[0], 4), "heavy": heavy, "parts": parts}
        row["eff"] = {k: round(row["s1"]["ms"] / (int(k[1:]) * row[k]["ms"]), 3) for k in ("s2", "s4", "s8")}
        print(json.dumps(row), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
