"""The split frame's two sides timed alone and together (round 5): with the split factor fixed
(RTX_SPLIT_FACTOR, no tuner), a serialized frame of the product build, of a build that launches
the main kernel only (RTX_ABL_CHAIN=1: the heavy tiles are not rendered) and of one that launches
the chain only (RTX_ABL_MAIN=1, except on the cost-measuring frames).  Critical-path bound: both ~
the larger alone; throughput bound: both ~ the sum.  Pixels of the ablated builds are wrong.
Usage (GPU box): python tools/chain_ablate.py <tag> [scene] [factor]"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
tag = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "Synthetic100k"
os.environ["RTX_SPLIT_FACTOR"] = sys.argv[3] if len(sys.argv) > 3 else "2.28"
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

W, H = (3840, 2160) if name == "Bunny8Lights" else (1920, 1080)
hs = HostScene(name)
s, cam = hs.view()
p = abi.make_params(W, H)
ctx = DeviceContext(0)
ctx.upload(s)
for _ in range(4):
    ctx.time_frames(cam, p, 16)
ms = min(ctx.time_frames(cam, p, 40) for _ in range(4))
print(f"{tag:10s} {name} {W}x{H} factor {os.environ['RTX_SPLIT_FACTOR']}: {ms:.4f} ms per frame, heavy {ctx.split_info()[0]}",
      flush=True)
ctx.close()
