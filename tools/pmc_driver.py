#!/usr/bin/env python3
"""Render one configuration F times for a rocprofv3 PMC pass (tools/pmc_configs.sh).

    python3 tools/pmc_driver.py <scene> <W> <H> <stripe_step> <frames>

Rank 0's stripes of a `stripe_step`-way tiled frame (16-row stripes; step 1 = the whole frame),
one frame at a time (synchronised), exactly the launches bench.py times: the first frame
measures tile costs, later ones run cost-ordered and split the heavy tiles."""
import ctypes as C
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402


# The split threshold the context's tuner converges to without a profiler (profiles/r05/
# split_tune_probe.txt).  Under PMC collection every dispatch is serialized, so the split chain
# can no longer run beside the main kernel and the tuner (which balances the two) would drift to
# its upper bound: the PMC runs fix the factor instead (RTX_SPLIT_FACTOR turns the tuner off).
TUNED_SPLIT_FACTOR = {"Synthetic100k": "2.0", "W4_Optional": "1.5"}


def main() -> int:
    scene, W, H, step, frames = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    factor = os.environ.setdefault("RTX_SPLIT_FACTOR", TUNED_SPLIT_FACTOR.get(scene, "1.5"))
    ctx = DeviceContext(0)
    hs = HostScene(scene)   # owns the arrays the view points into: keep it alive
    s, cam = hs.view()
    ctx.upload(s)
    p = abi.make_params(W, H, stripe_rows=16 if step > 1 else 0, stripe_first=0, stripe_step=step)
    for _ in range(frames):
        abi.check(ctx.lib.rtx_render_views_async(ctx.h, C.byref(cam), 1, C.byref(p), 0), "render", ctx.h)
        ctx.synchronize()
    heavy, parts = ctx.split_info()
    nb = C.c_uint64()
    abi.check(ctx.lib.rtx_scene_bytes(ctx.h, C.byref(nb)), "scene bytes", ctx.h)
    ctx.close()
    print(f"rendered {frames} frames of {scene} {W}x{H} stripe_step {step}")
    # (read by tools/pmc_configs.py: the per-phase algorithmic bytes)
    print(f"STATE heavy_tiles={heavy} parts={parts} scene_bytes={nb.value} lights={s.n_lights} "
          f"split_permille={int(round(float(factor) * 1000))}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
