"""Every BASELINE.json config (plus the other catalogue scenes) on one GPU, next to the
reference CPU Renderer built in place (oracle/_ref/ref_harness) on the same box's host.

GPU: kernel-only ms/frame (HIP events, min of 3 x `iters` launches), algorithmic FLOP of one
frame (instrumented kernel, SURVEY §8(d) model), end-to-end ms incl. the D2H copy of the
frame into pageable host memory; frames-in-flight throughput (2 render contexts, frames issued
round robin, as bench.py).  CPU: median Renderer::Render seconds over `frames` frames on
sched_getaffinity threads (the reference's hardware_concurrency), cgroup quota recorded.
Usage (GPU box):  python tools/config_table.py [out.json]
"""
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

sys.path.insert(0, str(ROOT))
from bench import FP32_PEAK_TFLOPS, cgroup_cpu_quota, write_obj_from_asset  # noqa: E402

COST = [41, 19, 14, 12, 63, 9, 15, 1, 26, 6, 31, 103]
CONFIGS = [  # (scene, W, H, cpu frames)
    ("W1", 640, 480, 8),
    ("W3", 1280, 720, 4),
    ("W4_Bunny", 1920, 1080, 4),
    ("W4_Reference", 1920, 1080, 4),
    ("W4_Optional", 1920, 1080, 2),
    ("Synthetic100k", 1920, 1080, 1),
    ("Bunny8Lights", 3840, 2160, 1),
]


def cpu_ref(harness, scene, W, H, threads, frames):
    with tempfile.TemporaryDirectory() as td:
        res = Path(td) / "Resources"
        res.mkdir()
        for a in abi.ASSET_DIR.glob("*.rtxmesh"):
            write_obj_from_asset(a, res / f"{a.stem}.obj")
        out = subprocess.run([str(harness), "bench", scene, "-1", str(W), str(H), str(threads), str(frames)],
                             cwd=td, check=True, capture_output=True, text=True, timeout=900)
    return json.loads(out.stdout.strip().splitlines()[-1])


def main():
    out_path = Path(sys.argv[1]) if len(sys.argv) > 1 else None
    # the reference's hardware_concurrency(): every CPU this process may run on; a cgroup quota
    # (the GPU box: 16 CPUs of 256) is recorded beside it
    threads = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    harness = ROOT / "oracle" / "_ref" / "ref_harness"
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    ctx = DeviceContext(0)
    ctx2 = DeviceContext(0)   # second frame in flight
    rows = []
    for scene, W, H, frames in CONFIGS:
        hs = HostScene(scene)
        s, cam = hs.view()
        ctx.upload(s)
        p = abi.make_params(W, H, 3, 1)
        ctx.time_frames(cam, p, 5)
        iters = 5 if scene == "Synthetic100k" else 50
        ms = min(ctx.time_frames(cam, p, iters) for _ in range(3))
        counts = ctx.count_work(cam, p)
        flop = int(sum(int(a) * b for a, b in zip(counts, COST)))
        host = np.zeros(W * H, np.uint32)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            abi.check(ctx.lib.rtx_render(ctx.h, C.byref(cam), C.byref(p), host.ctypes.data_as(C.POINTER(C.c_uint32)),
                                         None), "rtx_render", ctx.h)
            ts.append(time.perf_counter() - t0)
        e2e_ms = float(np.median(ts)) * 1e3
        # frames in flight: two contexts, frames issued round robin, wall time per frame
        ctx2.upload(s)
        pair = (ctx, ctx2)
        nfl = 10 if scene == "Synthetic100k" else 200
        for i in range(20):
            abi.check(ctx.lib.rtx_render_async(pair[i % 2].h, C.byref(cam), C.byref(p), 0), "render", ctx.h)
        ctx.synchronize(); ctx2.synchronize()
        t0 = time.perf_counter()
        for i in range(nfl):
            abi.check(ctx.lib.rtx_render_async(pair[i % 2].h, C.byref(cam), C.byref(p), 0), "render", ctx.h)
        ctx.synchronize(); ctx2.synchronize()
        fl_ms = (time.perf_counter() - t0) / nfl * 1e3
        row = {"scene": scene, "width": W, "height": H, "mode": "combined", "shadows": True,
               "kernel_ms": round(ms, 5), "mpix_s": round(W * H / (ms * 1e-3) / 1e6, 1),
               "flop_per_px": round(flop / (W * H), 1),
               "tflops": round(flop / (ms * 1e-3) / 1e12, 3),
               "frac_fp32": round(flop / (ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS, 4),
               "e2e_ms": round(e2e_ms, 4), "e2e_mpix_s": round(W * H / (e2e_ms * 1e-3) / 1e6, 1),
               "inflight2_ms": round(fl_ms, 5), "inflight2_mpix_s": round(W * H / (fl_ms * 1e-3) / 1e6, 1)}
        if harness.exists():
            r = cpu_ref(harness, scene, W, H, threads, frames)
            row.update({"cpu_mpix_s": round(r["mpix_s"], 3), "cpu_threads": threads, "cpu_frames": frames,
                        "cpu_fnv": r.get("fnv"), "speedup": round(row["mpix_s"] / r["mpix_s"], 1)})
        rows.append(row)
        print(json.dumps(row), flush=True)
    meta = {"cpu_model": cpu_model, "nproc": os.cpu_count(), "threads": threads, "cgroup_cpu_quota": quota,
            "rows": rows}
    if out_path:
        out_path.write_text(json.dumps(meta, indent=1))
    ctx.close()
    ctx2.close()


if __name__ == "__main__":
    main()
