"""Rank 0's share of a frame cut into 16-row stripes over s ranks, rendered with `k` frames in flight
(k contexts alternating, as bench.py's N-GPU frame mode runs a rank), wall time per frame, beside the
serialized time of one context.  For A/B of the schedule's concurrent (throughput) mode.
Usage: python tools/inflight_once.py <scene> <W> <H> <s> [k] [frames] [warm] [prior]
(prior 1: the contexts render the full frame first, serialized then in flight, as bench.py's predictor
does before the shares)"""
import ctypes as C
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

scene, W, H, st = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
k = int(sys.argv[5]) if len(sys.argv) > 5 else 2
frames = int(sys.argv[6]) if len(sys.argv) > 6 else 400
warm = int(sys.argv[7]) if len(sys.argv) > 7 else 2000
prior = len(sys.argv) > 8 and sys.argv[8] == "1"
hs = HostScene(scene)
s, cam = hs.view()
ctxs = [DeviceContext(0) for _ in range(k)]
for c in ctxs:
    c.upload(s)
p = abi.make_params(W, H, stripe_rows=16 if st > 1 else 0, stripe_first=0, stripe_step=st)


def run(n, p=p):
    t0 = time.perf_counter()
    for i in range(n):
        ctxs[i % k].render_async(cam, p)
    for c in ctxs:
        c.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


if prior:
    full = abi.make_params(W, H)
    ms = C.c_float()
    abi.check(ctxs[0].lib.rtx_time_views(ctxs[0].h, cam, 1, C.byref(full), 65, C.byref(ms)), "t", ctxs[0].h)
    run(240, full)
    print(f"  (full frame first: {run(200, full):.5f} ms with {k} in flight)")
run(warm)   # clocks up, schedules measured
best = min(run(frames) for _ in range(3))
ms = C.c_float()
abi.check(ctxs[0].lib.rtx_time_views(ctxs[0].h, cam, 1, C.byref(p), 200, C.byref(ms)), "t", ctxs[0].h)
print(f"{scene} {W}x{H} s={st}: {best:.5f} ms per frame with {k} in flight; serialized {ms.value:.5f}; "
      f"heavy {ctxs[0].split_info()[0]}, tune {ctxs[0].split_tune_info()}", flush=True)
for c in ctxs:
    c.close()
