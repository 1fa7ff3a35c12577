"""bench.py's strong-scaling predictor sequence on one scene, each in-flight share timed `reps` times in
a row (wall time per frame of 200 frames), to see how long a share's in-flight rate takes to settle.
Usage: python tools/predictor_probe.py <scene> <W> <H> [reps] [steps...]
PROBE_SPIN=n: n in-flight frames before each share's reps (PROBE_SPIN_OTHER=1: of the next share)."""
import ctypes as C
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

scene, W, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 4
steps = [int(x) for x in sys.argv[5:]] or [2, 4, 8]
SPIN = int(os.environ.get("PROBE_SPIN", "0"))             # in-flight frames before a share's reps
SPIN_OTHER = os.environ.get("PROBE_SPIN_OTHER", "0") == "1"   # ... of the next share instead
hs = HostScene(scene)
s, cam = hs.view()
ctxs = [DeviceContext(0) for _ in range(2)]
for c in ctxs:
    c.upload(s)
lib = ctxs[0].lib


def t(p, launches=30):
    ms = C.c_float()
    abi.check(lib.rtx_time_views(ctxs[0].h, C.byref(cam), 1, C.byref(p), 5, C.byref(ms)), "t", ctxs[0].h)
    best = 1e9
    for _ in range(2):
        abi.check(lib.rtx_time_views(ctxs[0].h, C.byref(cam), 1, C.byref(p), launches, C.byref(ms)), "t", ctxs[0].h)
        best = min(best, ms.value)
    return best


def inflight(p, frames=200):
    t0 = time.perf_counter()
    for i in range(frames):
        ctxs[i % 2].render_async(cam, p)
    for c in ctxs:
        c.synchronize()
    return (time.perf_counter() - t0) / frames * 1e3


full = abi.make_params(W, H)
print(f"full serialized {t(full):.5f}; in flight {[round(inflight(full), 5) for _ in range(reps)]}", flush=True)
for st in steps:
    ps = [abi.make_params(W, H, stripe_rows=16, stripe_first=r, stripe_step=st) for r in range(st)]
    ser = [round(t(p), 5) for p in ps]
    print(f"s={st} serialized {ser}", flush=True)
    for r, p in enumerate(ps):
        for c in ctxs:
            ms = C.c_float()
            abi.check(lib.rtx_time_views(c.h, C.byref(cam), 1, C.byref(p), 30, C.byref(ms)), "t", c.h)
        if SPIN:   # sustained in-flight load first: on another share (clock only) or this one
            inflight(ps[(r + 1) % st] if SPIN_OTHER else p, SPIN)
        print(f"  share {r}: in flight {[round(inflight(p), 5) for _ in range(reps)]}  "
              f"heavy {ctxs[0].split_info()[0]}/{ctxs[1].split_info()[0]} tune {ctxs[1].split_tune_info()['state']}",
              flush=True)
for c in ctxs:
    c.close()
