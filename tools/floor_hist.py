"""Per-work-item duration histograms of one stripe share (strong scaling's floor).

Diagnostic build only (per-wave start/end stamps, the walk itself unchanged):
    python tools/build_variant.py stamps_lean -DRTX_STAMPS=1 -DRTX_STAMPS_LEAN=1
    RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_stamps_lean.so \
        python tools/floor_hist.py <scene> <W> <H> [s ...]

A work item is one wave: a tile of the main launch (one piece, 64 rays) or one light part of a
split tile (the split launches).  For rank 0's share of a frame cut into 16-row stripes over s ranks
it prints one JSON line per s with
  frame_ms       rtx_time_views of this build (serialized launches, the predictor's method)
  span_us        first wave start to last wave end of the main launch
  waves          main-launch waves that rendered (split tiles' waves exit at once)
  hist           log2 histogram of main-launch wave durations: {"<lo>-<hi>us": count}
  max_wave_us    the longest single work item of the main launch, and where it started
  split_max_us   the longest split wave (any part), when tiles were split; split_p1/p2_max_us per phase
                 (P1 closest hit, P2 shadow rays: the chain runs them one after the other beside the main
                 launch, so frame_ms well above span_us means the chain is the share's critical path)
  ideal_us       sum of wave durations / resident wave slots (the share's perfect-balance time)
  floor_us       max(longest work item of either launch): no reordering of whole items finishes the
                 launch sooner, so span_us / floor_us near 1 says the share is at its floor
"""
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

lib = abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

SLOTS = int(os.environ.get("RTX_WAVE_SLOTS", str(256 * 4 * 8)))
PARTS = 1024   # kMaxParts
REPS = int(os.environ.get("FLOOR_REPS", "5"))
WORDS = 8      # kStampWords


def frame_ms(ctx, cam, p):
    ms = C.c_float()
    best = 1e9
    for _ in range(3):
        abi.check(ctx.lib.rtx_time_views(ctx.h, C.byref(cam), 1, C.byref(p), 40, C.byref(ms)), "time", ctx.h)
        best = min(best, ms.value)
    return best


def one(ctx, cam, W, H, st):
    p = abi.make_params(W, H, stripe_rows=16 if st > 1 else 0, stripe_first=0, stripe_step=st)
    for _ in range(30):   # clocks up, the schedule measured and settled (split tuner included)
        ctx.time_frames(cam, p, 40)
    fm = frame_ms(ctx, cam, p)
    heavy, nparts = ctx.split_info()
    cap = WORDS * ((W + 7) // 8) * ((H + 7) // 8) + 6 * PARTS
    buf = np.zeros(cap, np.uint64)
    nw = C.c_uint64()
    spans = []
    for _ in range(REPS):   # stamped frames back to back; the last one is kept
        buf[:] = 0
        abi.check(lib.rtx_debug_stamps(ctx.h, C.byref(cam), C.byref(p), buf.ctypes.data_as(C.POINTER(C.c_uint64)),
                                       cap, C.byref(nw)), "stamps", ctx.h)
        s = buf[: WORDS * nw.value].reshape(-1, WORDS)
        s = s[s[:, 1] > 0]
        spans.append(round(float(s[:, 1].max() - s[:, 0].min()) / 100.0, 1))
    s = buf[: WORDS * nw.value].reshape(-1, WORDS)
    s = s[s[:, 1] > 0]
    t0 = s[:, 0].min()
    start = (s[:, 0] - t0) / 100.0   # s_memrealtime: 100 MHz
    end = (s[:, 1] - t0) / 100.0
    dur = end - start
    edges = [0.0] + [2.0 ** k for k in range(0, 10)]
    hist = {}
    for lo, hi in zip(edges[:-1], edges[1:]):
        n = int(((dur >= lo) & (dur < hi)).sum())
        if n:
            hist[f"{lo:g}-{hi:g}us"] = n
    n_over = int((dur >= edges[-1]).sum())
    if n_over:
        hist[f">={edges[-1]:g}us"] = n_over
    split = buf[WORDS * nw.value: WORDS * nw.value + 6 * PARTS].reshape(2, PARTS, 3)
    split_max = float(split[:, :, 1].max()) / 100.0 if heavy else 0.0
    # per phase: P1 = closest hit over the parts, P2 = shadow rays over the parts (P3 shades, one wave a tile)
    phase_max = [round(float(split[k, :, 1].max()) / 100.0, 1) if heavy else 0.0 for k in range(2)]
    split_sum = float(split[:, :, 0].sum()) / 100.0 if heavy else 0.0
    w = int(dur.argmax())
    floor = max(float(dur.max()), split_max)
    ideal = (float(dur.sum()) + split_sum) / min(SLOTS, len(dur))
    return {"W": W, "H": H, "s": st, "frame_ms": round(fm, 5), "span_us": round(float(end.max()), 1), "spans_us": spans,
            "waves": int(len(dur)), "heavy_tiles": int(heavy), "hist": hist,
            "p50_us": round(float(np.median(dur)), 2), "p99_us": round(float(np.percentile(dur, 99)), 2),
            "max_wave_us": round(float(dur[w]), 1), "max_wave_start_us": round(float(start[w]), 1),
            "split_max_us": round(split_max, 1), "split_p1_max_us": phase_max[0], "split_p2_max_us": phase_max[1],
            "ideal_us": round(ideal, 1), "floor_us": round(floor, 1),
            "span_over_floor": round(float(end.max()) / floor, 3),
            "frame_over_floor": round(fm * 1e3 / floor, 3)}


def main():
    scene, W, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    steps = [int(x) for x in sys.argv[4:]] or [1, 4, 8]
    lib.rtx_debug_stamps.argtypes = [C.c_void_p, C.POINTER(abi.Camera), C.POINTER(abi.RenderParams),
                                     C.POINTER(C.c_uint64), C.c_uint64, C.POINTER(C.c_uint64)]
    hs = HostScene(scene)
    sc, cam = hs.view()
    for st in steps:
        ctx = DeviceContext(0)   # a fresh context per share: its own schedule
        try:
            ctx.upload(sc)
            print(json.dumps({"scene": scene, **one(ctx, cam, W, H, st)}), flush=True)
        finally:
            ctx.close()


if __name__ == "__main__":
    main()
