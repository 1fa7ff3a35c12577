"""Short-run behaviour of the headline frame (the driver times `bench.py --steps 20`):
per-frame GPU time of the first frames after an idle gap, and mean launch time of
short vs long bursts.  Usage: python tools/warmup_probe.py [scene W H]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "W4_Bunny"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
H = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
ctx = DeviceContext(0)
hs = HostScene(name)
s, cam = hs.view()
ctx.upload(s)
p = abi.make_params(W, H)
ctx.time_frames(cam, p, 5)
for idle_ms in (0, 2, 20, 200):
    ctx.time_frames(cam, p, 300)
    time.sleep(idle_ms / 1e3)
    per = [ctx.time_frames(cam, p, 1) * 1e3 for _ in range(12)]
    print(f"after {idle_ms:3d} ms idle, single frames (us): " + " ".join(f"{x:.1f}" for x in per), flush=True)
for idle_ms in (0, 20, 200):
    for n in (5, 20, 100, 1000):
        ctx.time_frames(cam, p, 300)
        time.sleep(idle_ms / 1e3)
        print(f"after {idle_ms:3d} ms idle, burst of {n:4d}: mean {ctx.time_frames(cam, p, n) * 1e3:.1f} us", flush=True)
ctx.close()
