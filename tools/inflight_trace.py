"""Rank 0's share with 2 frames in flight (2 contexts alternating), traced: every `chunk` frames the
wall time per frame, both contexts' heavy (split) tile counts and split factor / tuner state.
Usage: python tools/inflight_trace.py <scene> <W> <H> <s> [serial_warm] [frames] [chunk]
(serial_warm: serialized launches per context first, as bench.py's predictor does)"""
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
serial_warm = int(sys.argv[5]) if len(sys.argv) > 5 else 0
frames = int(sys.argv[6]) if len(sys.argv) > 6 else 4000
chunk = int(sys.argv[7]) if len(sys.argv) > 7 else 250
hs = HostScene(scene)
s, cam = hs.view()
ctxs = [DeviceContext(0) for _ in range(2)]
for c in ctxs:
    c.upload(s)
p = abi.make_params(W, H, stripe_rows=16 if st > 1 else 0, stripe_first=0, stripe_step=st)
if serial_warm:
    for c in ctxs:
        ms = C.c_float()
        abi.check(c.lib.rtx_time_views(c.h, C.byref(cam), 1, C.byref(p), serial_warm, C.byref(ms)), "t", c.h)
    print(f"after {serial_warm} serialized: heavy {[c.split_info()[0] for c in ctxs]} "
          f"tune {[c.split_tune_info() for c in ctxs]}", flush=True)
i = 0
while i < frames:
    t0 = time.perf_counter()
    calls = []
    for _ in range(chunk):
        tc = time.perf_counter()
        ctxs[i % 2].render_async(cam, p)
        calls.append(time.perf_counter() - tc)
        i += 1
    for c in ctxs:
        c.synchronize()
    dt = (time.perf_counter() - t0) / chunk * 1e3
    calls = sorted(calls)
    tu = [c.split_tune_info() for c in ctxs]
    print(f"frames {i:5d}: {dt:.5f} ms/frame  heavy {[c.split_info()[0] for c in ctxs]}  "
          f"factor {[round(x['factor'], 3) for x in tu]} {[x['state'] for x in tu]}  host call us "
          f"p50 {calls[len(calls) // 2] * 1e6:.1f} p90 {calls[len(calls) * 9 // 10] * 1e6:.1f} "
          f"max {calls[-1] * 1e6:.1f}  probe {[c.inflight_info() for c in ctxs]}", flush=True)
for c in ctxs:
    c.close()
