#!/usr/bin/env python3
"""Headline benchmark of the HIP render path (BASELINE.json metric):
Mpixels/s (primary + shadow rays) at 1920x1080 on Scene_W4_BunnyScene (Initialize
state, Combined lighting, shadows on).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step renders one batch: N views of the Bunny scene (view f = the reference camera
moved 0.05*f along x), each 1920x1080, cut into 16-row stripes dealt round-robin over
the N ranks (rank r renders view f's stripes s with s % N == (r - f) mod N).  Every
rank therefore renders exactly one frame's worth of pixels per step (weak scaling); at
N = 1 a step is exactly one reference frame.  The ranks share no data: there is no
collective on the data path, only a gloo barrier / max-reduce of the timings.

Inputs are resident in HBM before timing (scene uploaded once); the output frame stays
in HBM.  Prints ONE JSON line on rank 0.

Frames in flight (--inflight, default 2): consecutive steps are issued round robin to
that many render contexts on the rank's GPU (each its own stream, frame buffer and tile
schedule), so frame k+1 starts while frame k's last waves drain instead of after the
inter-kernel gap — a renderer's frame pipelining; every frame is rendered in full inside
the timed region.  `roofline.kernel_ms` is the serialized launch time of ONE context
(HIP events on its stream), the figure a rocprofv3 kernel trace of `--inflight 1` shows.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import struct
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

# Load the HIP library before anything else can pull in another copy of the runtime.
from gp1_raytracer_2223_amd import abi  # noqa: E402

abi.load_hip()
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

FP32_PEAK_TFLOPS = 157.3   # MI355X FP32 vector peak (MI355X_MICROARCH.md, spec)
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak (spec)


def make_views(cam: abi.Camera, n: int) -> "C.Array":
    arr = (abi.Camera * n)()
    for f in range(n):
        C.memmove(C.byref(arr[f]), C.byref(cam), C.sizeof(abi.Camera))
        arr[f].origin[0] = cam.origin[0] + 0.05 * f
    return arr


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist   # control plane only (gloo): no data-path collective
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # gloo prints its connection log on stdout; keep stdout for the one JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
                dist.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def write_obj_from_asset(asset: Path, out_obj: Path) -> None:
    """Re-emit an .rtxmesh as OBJ text (exact float round trip, 1-based faces) so the
    reference harness can load it where /root/reference does not exist."""
    b = asset.read_bytes()
    nv, ni = struct.unpack_from("<II", b, 4)
    pos = np.frombuffer(b, np.float32, 3 * nv, 12).reshape(-1, 3)
    idx = np.frombuffer(b, np.int32, ni, 12 + 12 * nv).reshape(-1, 3)
    lines = [f"v {x:.9g} {y:.9g} {z:.9g}" for x, y, z in pos.tolist()]
    lines += [f"f {a + 1} {b_ + 1} {c + 1}" for a, b_, c in idx.tolist()]
    out_obj.write_text("\n".join(lines) + "\n")


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def cpu_baseline(scene: str, width: int, height: int, frames: int) -> dict | None:
    """The reference CPU Renderer timed on this host (rank 0, N = 1 only): the
    reference's own sources built in place by oracle/ref (kind "reference"), or the C
    restatement in oracle/ when that build is absent (kind "port")."""
    threads = min(16, os.cpu_count() or 1)
    harness = ROOT / "oracle" / "_ref" / "ref_harness"
    if harness.exists():
        with tempfile.TemporaryDirectory() as td:
            res = Path(td) / "Resources"
            res.mkdir()
            for stem in ("lowpoly_bunny2", "Assignment3D1"):
                write_obj_from_asset(abi.ASSET_DIR / f"{stem}.rtxmesh", res / f"{stem}.obj")
            out = subprocess.run([str(harness), "bench", scene, "-1", str(width), str(height), str(threads),
                                  str(frames)], cwd=td, check=True, capture_output=True, text=True, timeout=600)
            r = json.loads(out.stdout.strip().splitlines()[-1])
            # one frame on one core as well (BASELINE.md §3 records both)
            one = subprocess.run([str(harness), "bench", scene, "-1", str(width), str(height), "1", "1"], cwd=td,
                                 check=True, capture_output=True, text=True, timeout=600)
            r1 = json.loads(one.stdout.strip().splitlines()[-1])
        return {"value": round(r["mpix_s"], 4), "unit": "Mpixels/s", "cores": threads, "kind": "reference",
                "sample": f"{frames} frames of {scene} {width}x{height} (median of Renderer::Render, "
                          f"reference sources built with g++ -O2 -ffp-contract=off, {threads} threads, "
                          f"1024-pixel dynamic chunks)", "median_s": r["median_s"], "fnv": r["fnv"],
                "single_thread_mpix_s": round(r1["mpix_s"], 4), "cpu_model": cpu_model(),
                "nproc": os.cpu_count()}
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_bind   # test infrastructure: the checker, timed here as the CPU baseline
    hs = HostScene(scene)
    s, cam = hs.view()
    p = abi.make_params(width, height)
    oracle_bind.render(s, cam, p, threads=threads, want_rgb=False)
    ts = []
    for _ in range(frames):
        t0 = time.perf_counter()
        oracle_bind.render(s, cam, p, threads=threads, want_rgb=False)
        ts.append(time.perf_counter() - t0)
    med = float(np.median(ts))
    return {"value": round(width * height / med / 1e6, 4), "unit": "Mpixels/s", "cores": threads, "kind": "port",
            "sample": f"{frames} frames of {scene} {width}x{height} (median, C restatement oracle/rtx_oracle.c, "
                      f"{threads} threads)", "median_s": med}


def pmc_traffic(scene: str, width: int, height: int, views: int) -> tuple[int | None, str | None]:
    """HBM bytes per launch of the render kernel from the committed rocprofv3 PMC summary of
    this same command (tools/profile.sh -> profiles/r01/pmc_summary.json: 2 x FETCH_SIZE +
    WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md), when the configuration
    matches.  A benchmark process cannot read its own PMC counters, so this is the
    profiled value, not a live one."""
    f = ROOT / "profiles" / "r01" / "pmc_summary.json"
    try:
        d = json.loads(f.read_text())
    except (OSError, ValueError):
        return None, None
    if d.get("config") != {"scene": scene, "width": width, "height": height, "views": views}:
        return None, None
    return int(d["hbm_bytes_per_launch"]), str(f.relative_to(ROOT))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--scene", default="W4_Bunny")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--cpu-frames", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inflight", type=int, default=2, help="frames in flight (render contexts per GPU)")
    args = ap.parse_args()

    # The render contexts come up BEFORE the gloo process group: torch's gloo barrier
    # initialises torch's own bundled HIP runtime, after which this process's ROCm runtime
    # (librtx_hip) no longer detects the device ("no ROCm-capable device", seen at N = 2).
    # RTX_BENCH_DEVICE pins every rank to one device: rehearsing the N-rank path on a
    # one-GPU machine (the driver's multi-GPU runs leave it unset: rank r -> device LOCAL_RANK)
    dev = int(os.environ.get("RTX_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    ctxs = [DeviceContext(dev) for _ in range(max(1, args.inflight))]
    d = Dist()
    N = d.world
    if args.gpus != N and d.rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={N}; using {N}", file=sys.stderr)
    hs = HostScene(args.scene)
    scene, cam = hs.view()
    for c in ctxs:
        c.upload(scene)
    ctx = ctxs[0]
    views = make_views(cam, N)
    params = abi.make_params(args.width, args.height, stripe_rows=16 if N > 1 else 0,
                             stripe_first=d.rank, stripe_step=N)
    lib = ctx.lib

    def step(i):
        c = ctxs[i % len(ctxs)]
        rc = lib.rtx_render_views_async(c.h, views, N, C.byref(params), 0)
        if rc != abi.RTX_OK:
            abi.check(rc, "rtx_render_views_async", c.h)

    def sync_all():
        for c in ctxs:
            c.synchronize()

    for i in range(args.warmup):
        step(i)
    sync_all()

    d.barrier()
    sync_all()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    sync_all()
    d.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = d.max(elapsed)

    # Kernel-only time of the same launches, HIP events on the launch stream.
    kernel_ms = C.c_float()
    abi.check(lib.rtx_time_views(ctx.h, views, N, C.byref(params), args.steps, C.byref(kernel_ms)),
              "rtx_time_views", ctx.h)
    kernel_ms = kernel_ms.value

    # Algorithmic work of one launch (SURVEY §8(d) FLOP model) from the instrumented kernel.
    flop = 0
    counts_total = np.zeros(12, np.uint64)
    for f in range(N):
        pv = abi.make_params(args.width, args.height, stripe_rows=16 if N > 1 else 0,
                             stripe_first=(d.rank - f) % N, stripe_step=N)
        counts_total += ctx.count_work(views[f], pv)
    cost = [41, 19, 14, 12, 63, 9, 15, 1, 26, 6, 31, 103]
    flop = int(sum(int(c) * w for c, w in zip(counts_total, cost)))
    pixels_per_rank = int(counts_total[0])

    # End-to-end single frame incl. D2H of the full frame into host memory (not `value`).
    e2e = None
    if N == 1:
        host = np.zeros(args.width * args.height, np.uint32)
        p1 = abi.make_params(args.width, args.height)
        ts = []
        for _ in range(10):
            t1 = time.perf_counter()
            abi.check(lib.rtx_render(ctx.h, C.byref(cam), C.byref(p1), host.ctypes.data_as(C.POINTER(C.c_uint32)),
                                     None), "rtx_render", ctx.h)
            ts.append(time.perf_counter() - t1)
        e2e = args.width * args.height / float(np.median(ts)) / 1e6

    cpu = None
    if d.rank == 0 and N == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args.scene, args.width, args.height, args.cpu_frames)
        except Exception as e:   # the baseline must not take the headline down
            cpu = {"value": None, "unit": "Mpixels/s", "cores": 0, "kind": "reference", "sample": f"failed: {e}"}

    ms_per_step = elapsed / args.steps * 1e3
    total_pixels = N * args.width * args.height * args.steps
    value = total_pixels / elapsed / 1e6
    achieved = flop / (kernel_ms * 1e-3) / 1e12 if kernel_ms > 0 else 0.0
    traffic, traffic_src = pmc_traffic(args.scene, args.width, args.height, N)
    out = {
        "metric": "Mpixels/s (primary+shadow rays) at 1920x1080; per-channel max-abs vs CPU ref",
        "value": round(value, 3),
        "unit": "Mpixels/s",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic camera views of the reference Scene_W4_BunnyScene (lowpoly_bunny2.obj, 292 tris, "
                "3 point lights, Initialize state); no datasets",
        "config": {"workload": f"{args.scene} {args.width}x{args.height}, Combined lighting, shadows on, "
                               f"{N} view(s) per step striped over {N} rank(s)",
                   "scene": args.scene, "width": args.width, "height": args.height, "views_per_step": N,
                   "stripe_rows": 16 if N > 1 else 0, "parallelism": f"image stripes x{N} (no collective)",
                   "frames_in_flight": len(ctxs)},
        "roofline": {"bound": "valu", "achieved": round(achieved, 4), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / FP32_PEAK_TFLOPS, 5), "traffic": traffic,
                     "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": traffic_src,
                     "hbm_gbs": round(traffic / (kernel_ms * 1e-3) / 1e9, 2) if traffic and kernel_ms > 0 else None,
                     # north star: the HBM roofline fraction, reported beside the VALU one
                     "hbm_frac": round(traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                     if traffic and kernel_ms > 0 else None,
                     "kernel": "rtx_render_kernel<false, 0> (+ split phases 1-3 when tiles are heavy)", "kernel_ms": round(kernel_ms, 5),
                     "flop_per_launch": flop, "pixels_per_launch": pixels_per_rank,
                     "flop_per_pixel": round(flop / max(pixels_per_rank, 1), 2),
                     "note": "FP32 VALU-bound path (no dense contraction, 4 B/pixel of HBM output); "
                             "FLOP = SURVEY §8(d) algorithmic model counted by the instrumented kernel"},
        "cpu_baseline": cpu,
        "end_to_end_mpix_s": round(e2e, 3) if e2e else None,
    }
    if cpu and cpu.get("value"):
        out["speedup_vs_cpu"] = round(value / cpu["value"], 1)
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()
    d.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
