"""Heavy-tile split rendering probe: heavy-tile count, parts, frame time with split on/off.
Usage: python tools/split_probe.py [scene W H]  (run under rocprofv3 --kernel-trace for phases)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "Synthetic100k"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
H = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
ctx = DeviceContext(0)
hs = HostScene(name)
s, cam = hs.view()
ctx.upload(s)
p = abi.make_params(W, H, 3, 1)
ctx.time_frames(cam, p, 2)
heavy, parts = ctx.split_info()
ms = min(ctx.time_frames(cam, p, 5) for _ in range(2))
print(f"{name} {W}x{H}: heavy tiles {heavy} of {((W + 15) // 16) * ((H + 15) // 16)}, parts {parts}, "
      f"frame {ms:.3f} ms", flush=True)
