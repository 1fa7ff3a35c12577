#!/usr/bin/env python3
"""Headline benchmark of the HIP render path (BASELINE.json metric):
Mpixels/s (primary + shadow rays) at 1920x1080 on Scene_W4_BunnyScene (Initialize
state, Combined lighting, shadows on).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scene S --width W --height H]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step renders N views of the scene (`--mode views`, the default): view f is the reference
camera moved 0.05 f along x, and every view's rows are cut into 16-row stripes dealt round
robin over the N ranks (rank r owns view f's stripe s iff s % N == (r - f) mod N; SURVEY
§8(e)), so every image is tiled across all the GPUs and every rank renders one frame's
worth of pixels per step — weak scaling, the sharding rule for a path of independent
pixels.  At N = 1 a step is exactly one reference Renderer::Render frame.  `--mode frame`
tiles ONE frame per step over the N ranks (strong scaling: each rank renders 1/N of a
frame, so at 8 GPUs a 1080p frame no longer fills a GPU).

Two timed regions, each bracketed by barrier + stream sync and max-reduced over ranks:
  1. `value`: K steps with inputs resident in HBM and the frames left in HBM (the
     metric's device throughput);
  2. `host_gather`: K steps whose frames are ALSO gathered into page-locked host frames
     shared by all ranks (/dev/shm mapping, hipHostRegister; every rank hipMemcpy2DAsync's
     only its own stripes over its own PCIe link) — the north star's "independent tiles
     gathered on host".  PCIe-inclusive, so never `value`.
No collective on the data path: the ranks' only exchange is a gloo barrier and the
max-reduce of the timings.

Frames in flight (--inflight, default 2): consecutive steps go round robin to that many
render contexts on the rank's GPU (each its own stream, frame buffer and tile schedule),
so frame k+1 starts while frame k's last waves drain.  `roofline.kernel_ms` is the
serialized launch time of ONE context (HIP events on its stream, mean of 1000 launches), the
figure a rocprofv3 kernel trace of `--inflight 1` shows.  It is measured first, before the W
warm-up steps: those 1000 launches (~60 ms) also take the GPU from its idle clock to its
steady rendering clock, which a short run's few warm-up steps do not.

After timing, the gathered frame is checked against the reference: `parity` carries the
SHA-256 comparison with tests/golden/config_<scene>_<W>x<H>.npz (the frame the reference
built in place produced), the max-abs of the float colour on the golden's 4096 samples,
and the frame's FNV beside `cpu_baseline.fnv` (the reference timed in this same run).
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
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
from gp1_raytracer_2223_amd.hostframe import SharedFrame  # noqa: E402
from gp1_raytracer_2223_amd.renderer import DeviceContext  # noqa: E402
from gp1_raytracer_2223_amd.scene import HostScene  # noqa: E402

FP32_PEAK_TFLOPS = 157.3   # MI355X FP32 vector peak (MI355X_MICROARCH.md, spec)
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak (spec)
GOLDEN = ROOT / "tests" / "golden"
# ref_harness's FNV-1a (oracle/ref/ref_harness.cpp `bench`) starts from the decimal basis
# 1469598103934665603; SURVEY §8(c)'s recorded hashes use the same one.
FNV_BASIS = 1469598103934665603
COST = [41, 19, 14, 12, 63, 9, 15, 1, 26, 6, 31, 103]   # SURVEY §8(d) FLOP per counted unit


def make_views(cam: abi.Camera, n: int) -> "C.Array":
    arr = (abi.Camera * n)()
    for f in range(n):
        C.memmove(C.byref(arr[f]), C.byref(cam), C.sizeof(abi.Camera))
        arr[f].origin[0] = cam.origin[0] + 0.05 * f
    return arr


def fnv1a(px: np.ndarray) -> str:
    h = FNV_BASIS
    m = (1 << 64) - 1
    for b in np.ascontiguousarray(px, dtype="<u4").view(np.uint8).tobytes():
        h = ((h ^ b) * 0x100000001B3) & m
    return f"{h:016x}"


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
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

    def sum_i64(self, xs: list[int]) -> list[int]:
        if self.world == 1:
            return xs
        import torch
        t = torch.tensor(xs, dtype=torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return [int(v) for v in t.tolist()]

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


def cgroup_cpu_quota() -> float | None:
    """CPUs this process may use per the cgroup-v2 quota (cpu.max), None if unlimited."""
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else int(q) / int(period)
    except (OSError, ValueError):
        return None


def cpu_baseline(scene: str, width: int, height: int, frames: int) -> dict | None:
    """The reference CPU Renderer timed on this host (rank 0, N = 1 only): the
    reference's own sources built in place by oracle/ref (kind "reference"), or the C
    restatement in oracle/ when that build is absent (kind "port").

    Threads = every CPU this process may run on (len(sched_getaffinity)), which is what
    the reference's PPL parallel_for uses (std::thread::hardware_concurrency, Renderer.cpp:
    79-85).  Where a cgroup CPU quota caps the process below that (the GPU box: 16 CPUs of
    256), the quota-sized run and a single-thread run are recorded too, and
    `full_host_upper_bound` = single-thread rate x hardware threads (perfect linear
    scaling over every hardware thread, SMT included) bounds what the whole host could do."""
    nthreads = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    harness = ROOT / "oracle" / "_ref" / "ref_harness"
    runs = {}
    if harness.exists():
        with tempfile.TemporaryDirectory() as td:
            res = Path(td) / "Resources"
            res.mkdir()
            for stem in ("lowpoly_bunny2", "Assignment3D1"):
                write_obj_from_asset(abi.ASSET_DIR / f"{stem}.rtxmesh", res / f"{stem}.obj")

            def run(threads, nframes):
                out = subprocess.run([str(harness), "bench", scene, "-1", str(width), str(height), str(threads),
                                      str(nframes)], cwd=td, check=True, capture_output=True, text=True, timeout=900)
                return json.loads(out.stdout.strip().splitlines()[-1])
            runs["all"] = run(nthreads, frames)
            if quota is not None and int(quota) < nthreads:
                runs["quota"] = run(max(1, int(quota)), frames)
            runs["one"] = run(1, 1)
        kind = "reference"
        how = "reference sources built in place with g++ -O2 -ffp-contract=off (oracle/ref), 1024-pixel dynamic chunks"
    else:
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_bind   # test infrastructure: the checker, timed here as the CPU baseline
        hs = HostScene(scene)
        s, cam = hs.view()
        p = abi.make_params(width, height)

        def run(threads, nframes):
            oracle_bind.render(s, cam, p, threads=threads, want_rgb=False)
            ts = []
            for _ in range(nframes):
                t0 = time.perf_counter()
                oracle_bind.render(s, cam, p, threads=threads, want_rgb=False)
                ts.append(time.perf_counter() - t0)
            med = float(np.median(ts))
            return {"median_s": med, "mpix_s": width * height / med / 1e6, "fnv": None}
        runs["all"] = run(nthreads, frames)
        if quota is not None and int(quota) < nthreads:
            runs["quota"] = run(max(1, int(quota)), frames)
        runs["one"] = run(1, 1)
        kind = "port"
        how = "C restatement oracle/rtx_oracle.c"
    r = runs["all"]
    one = runs["one"]["mpix_s"]
    out = {"value": round(r["mpix_s"], 4), "unit": "Mpixels/s", "cores": nthreads, "kind": kind,
           "sample": f"{frames} frames of {scene} {width}x{height}, median of Renderer::Render, {nthreads} threads "
                     f"(= sched_getaffinity, the reference's hardware_concurrency), {how}",
           "median_s": r["median_s"], "fnv": r.get("fnv"),
           "single_thread_mpix_s": round(one, 4),
           "full_host_upper_bound_mpix_s": round(one * nthreads, 2),
           "cpu_model": cpu_model(), "nproc": os.cpu_count(), "cgroup_cpu_quota": quota}
    if "quota" in runs:
        out["quota_threads_mpix_s"] = round(runs["quota"]["mpix_s"], 4)
        out["note"] = (f"this process is capped by a cgroup quota of {quota:g} CPUs, so the {nthreads}-thread run "
                       f"gets at most {quota:g} CPUs of time; full_host_upper_bound_mpix_s assumes perfect scaling "
                       f"of the single-thread rate to all {nthreads} hardware threads")
    return out


def pmc_traffic(scene: str, width: int, height: int, views: int) -> tuple[int | None, str | None]:
    """HBM bytes per launch of the render kernel from the newest committed rocprofv3 PMC
    summary of this same configuration (tools/profile.sh -> profiles/r*/pmc_summary.json:
    2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md).  A benchmark
    process cannot read its own PMC counters, so this is the profiled value, not a live one."""
    for f in sorted(ROOT.glob("profiles/r*/pmc_summary.json"), reverse=True):
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        if d.get("config") == {"scene": scene, "width": width, "height": height, "views": views}:
            return int(d["hbm_bytes_per_launch"]), str(f.relative_to(ROOT))
    return None, None


def golden_for(scene: str, width: int, height: int):
    f = GOLDEN / f"config_{scene}_{width}x{height}.npz"
    return (np.load(f), f) if f.exists() else (None, None)


def parity_report(px: np.ndarray, rgb: np.ndarray, scene: str, width: int, height: int, cpu: dict | None) -> dict:
    """Self-check of the benchmarked frame against the reference's own frame."""
    g, f = golden_for(scene, width, height)
    out = {"frame": "the host-gathered frame of the timed contexts (cost-ordered / split state)",
           "gpu_fnv": fnv1a(px)}
    if cpu and cpu.get("fnv"):
        out["cpu_fnv"] = cpu["fnv"]
        out["fnv_match"] = out["gpu_fnv"] == cpu["fnv"]
    if g is None:
        out["reference"] = None
        return out
    rgb3 = rgb.reshape(-1, 3)
    idx = g["idx"]
    ch = lambda p: np.stack([(p >> 16) & 255, (p >> 8) & 255, p & 255], -1).astype(np.int32)  # noqa: E731
    px_ok = hashlib.sha256(px.tobytes()).hexdigest() == str(g["sha_pixels"][0])
    rgb_ok = hashlib.sha256(rgb3.tobytes()).hexdigest() == str(g["sha_rgb"][0])
    out.update({"reference": str(f.relative_to(ROOT)), "pixels_sha256_match": px_ok, "rgb_sha256_match": rgb_ok,
                "bit_exact": bool(px_ok and rgb_ok),
                "max_abs": float(np.abs(rgb3[idx] - g["rgb"]).max()),
                "max_lsb": int(np.abs(ch(px[idx]) - ch(g["pixels"])).max()),
                "samples": int(idx.size), "tolerance": "max_abs <= 1e-4, <= 1 LSB (north star)"})
    out["within_tolerance"] = bool(out["max_abs"] <= 1e-4 and out["max_lsb"] <= 1)
    return out


K_KERNEL_LAUNCHES = 1000   # launches averaged for roofline.kernel_ms


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--scene", default="W4_Bunny")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--mode", choices=["frame", "views"], default="views",
                    help="frame: one frame per step tiled over the ranks (strong); views: N views per step (weak)")
    ap.add_argument("--cpu-frames", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true", help="skip the host-gather timed region")
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
    lib = ctx.lib
    W, H = args.width, args.height
    striped = N > 1
    if args.mode == "frame":
        nviews = 1
        views = make_views(cam, 1)
        params = abi.make_params(W, H, stripe_rows=16 if striped else 0, stripe_first=d.rank, stripe_step=N)
        frame_pixels = W * H                       # one frame per step, all ranks together
    else:
        nviews = N
        views = make_views(cam, N)
        params = abi.make_params(W, H, stripe_rows=16 if striped else 0, stripe_first=d.rank, stripe_step=N)
        frame_pixels = N * W * H                   # N frames per step, one frame's worth per rank

    def step(i, gather_to=None):
        c = ctxs[i % len(ctxs)]
        rc = lib.rtx_render_views_async(c.h, views, nviews, C.byref(params), 0)
        if rc != abi.RTX_OK:
            abi.check(rc, "rtx_render_views_async", c.h)
        if gather_to is not None:
            c.gather_async(gather_to)

    def sync_all():
        for c in ctxs:
            c.synchronize()

    def timed(fn, k):
        d.barrier()
        sync_all()
        t0 = time.perf_counter()
        for i in range(k):
            fn(i)
        sync_all()
        d.barrier()
        return d.max(time.perf_counter() - t0)

    # Kernel-only time of the same launches (HIP events on the launch stream), the roofline's
    # denominator: the mean of kKernelLaunches serialized launches, taken first — it also brings
    # the GPU from its idle clock to the steady rendering clock (profiles/r02/warmup_probe.txt),
    # which the requested W warm-up steps alone (the driver uses 5) do not.
    kernel_ms = C.c_float()
    abi.check(lib.rtx_time_views(ctx.h, views, nviews, C.byref(params), K_KERNEL_LAUNCHES,
                                 C.byref(kernel_ms)), "rtx_time_views", ctx.h)
    kernel_ms = kernel_ms.value

    for i in range(args.warmup):
        step(i)
    sync_all()

    # ---- timed region 1: device-resident frames (`value`)
    elapsed = timed(step, args.steps)

    # ---- timed region 2: the same frames gathered into host frames shared by the ranks
    shared = None
    gathered = None
    nbytes = nviews * W * H * 16    # uint32 pixels + float RGB plane per view (parity check)
    tag = f"{os.environ.get('MASTER_PORT', 'solo')}_{os.getuid()}_{os.getppid() if N > 1 else os.getpid()}"
    if d.rank == 0:
        shared = SharedFrame.create(tag, nbytes)
    d.barrier()
    if d.rank != 0:
        shared = SharedFrame.attach(tag, nbytes)
    d.barrier()
    if d.rank == 0:
        shared.unlink()   # every rank has it mapped: nothing stays behind in /dev/shm
    pinned = shared.pin(ctx)
    host_px = shared.view(np.uint32, nviews * W * H)
    host_rgb = shared.view(np.float32, 3 * nviews * W * H, offset=4 * nviews * W * H)
    if not args.no_gather:
        for i in range(min(args.warmup, 10)):
            step(i, host_px)
        sync_all()
        g_elapsed = timed(lambda i: step(i, host_px), args.steps)
        gathered = {"mpix_s": round(frame_pixels * args.steps / g_elapsed / 1e6, 3),
                    "ms_per_step": round(g_elapsed / args.steps * 1e3, 5), "pinned": bool(pinned),
                    "target": "page-locked host frames (one per view) shared by all ranks (/dev/shm mapping)",
                    "copy": "hipMemcpy2DAsync of the rank's own 16-row stripes (rtx_gather_async)"}

    # Algorithmic work of one launch (SURVEY §8(d) FLOP model) from the instrumented kernel.
    counts_total = np.zeros(12, np.uint64)
    for f in range(nviews):
        pv = abi.make_params(W, H, stripe_rows=16 if striped else 0,
                             stripe_first=(d.rank - f) % N if args.mode == "views" else d.rank, stripe_step=N)
        counts_total += ctx.count_work(views[f], pv)
    flop = int(sum(int(c) * w for c, w in zip(counts_total, COST)))
    pixels_per_rank = int(counts_total[0])
    frame_flop, frame_counted = d.sum_i64([flop, pixels_per_rank])

    # Parity of the benchmarked frame: every rank renders its stripes once more on the timed
    # context (same schedule state), with colours, gathered into the shared host frame.
    parity = None
    if shared is not None:
        abi.check(lib.rtx_render_views_async(ctx.h, views, nviews, C.byref(params), 1), "rtx_render_views_async",
                  ctx.h)
        ctx.gather_async(host_px, host_rgb)
        ctx.synchronize()
        d.barrier()

    # End-to-end single frame through the blocking C-ABI entry into pageable memory (N = 1).
    e2e = None
    if N == 1:
        host = np.zeros(W * H, np.uint32)
        p1 = abi.make_params(W, H)
        ts = []
        for _ in range(10):
            t1 = time.perf_counter()
            abi.check(lib.rtx_render(ctx.h, C.byref(cam), C.byref(p1), host.ctypes.data_as(C.POINTER(C.c_uint32)),
                                     None), "rtx_render", ctx.h)
            ts.append(time.perf_counter() - t1)
        e2e = W * H / float(np.median(ts)) / 1e6

    cpu = None
    if d.rank == 0 and N == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args.scene, W, H, args.cpu_frames)
        except Exception as e:   # the baseline must not take the headline down
            cpu = {"value": None, "unit": "Mpixels/s", "cores": 0, "kind": "reference", "sample": f"failed: {e}"}
    if d.rank == 0 and shared is not None:
        # view 0 is the reference camera: the frame the goldens were made from
        parity = parity_report(np.array(host_px[:W * H]), np.array(host_rgb[:3 * W * H]), args.scene, W, H, cpu)

    ms_per_step = elapsed / args.steps * 1e3
    value = frame_pixels * args.steps / elapsed / 1e6
    achieved = flop / (kernel_ms * 1e-3) / 1e12 if kernel_ms > 0 else 0.0
    traffic, traffic_src = pmc_traffic(args.scene, W, H, nviews) if not striped else (None, None)
    strong = args.mode == "frame"
    out = {
        "metric": "Mpixels/s (primary+shadow rays) at 1920x1080; per-channel max-abs vs CPU ref",
        "value": round(value, 3),
        "unit": "Mpixels/s",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic: the reference's {args.scene} scene (Initialize state) built by the host scene layer; "
                "no datasets",
        "config": {"workload": (f"{args.scene} {W}x{H}, Combined lighting, shadows on, one frame per step"
                                if N == 1 else
                                f"{args.scene} {W}x{H}, Combined lighting, shadows on, one frame per step tiled "
                                f"over {N} ranks in 16-row stripes" if strong else
                                f"{args.scene} {W}x{H}, Combined lighting, shadows on, {N} views per step, each "
                                f"tiled over the {N} ranks in 16-row stripes"),
                   "scene": args.scene, "width": W, "height": H, "views_per_step": nviews,
                   "stripe_rows": 16 if striped else 0,
                   "parallelism": f"image stripes x{N} (no collective)", "frames_in_flight": len(ctxs)},
        "roofline": {"bound": "valu", "achieved": round(achieved, 4), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / FP32_PEAK_TFLOPS, 5), "traffic": traffic,
                     "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": traffic_src,
                     "hbm_gbs": round(traffic / (kernel_ms * 1e-3) / 1e9, 2) if traffic and kernel_ms > 0 else None,
                     # north star: the HBM roofline fraction, reported beside the VALU one
                     "hbm_frac": round(traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                     if traffic and kernel_ms > 0 else None,
                     "kernel": "rtx_render_kernel<false, 0, false, SPEC> (the specialised variant the scene's "
                               "facts select; + split phases 1-3 when tiles are heavy)",
                     "kernel_ms": round(kernel_ms, 5), "kernel_launches": K_KERNEL_LAUNCHES,
                     "flop_per_launch": flop, "pixels_per_launch": pixels_per_rank,
                     "flop_per_pixel": round(flop / max(pixels_per_rank, 1), 2),
                     "frame_flop_all_ranks": frame_flop, "frame_pixels_counted": frame_counted,
                     "note": "FP32 VALU-bound path (no dense contraction, 4 B/pixel of HBM output); "
                             "FLOP = SURVEY §8(d) algorithmic model counted by the instrumented kernel; "
                             "kernel_ms/achieved are rank 0's launches (mean of kernel_launches serialized launches, "
                             "timed before the warm-up)"},
        "cpu_baseline": cpu,
        "parity": parity,
        "host_gather": gathered,
        "end_to_end_mpix_s": round(e2e, 3) if e2e else None,
    }
    if cpu and cpu.get("value"):
        out["speedup_vs_cpu"] = round(value / cpu["value"], 1)
        if cpu.get("full_host_upper_bound_mpix_s"):
            out["speedup_vs_cpu_full_host_upper_bound"] = round(value / cpu["full_host_upper_bound_mpix_s"], 1)
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    if shared is not None:
        shared.close()
    for c in ctxs:
        c.close()
    d.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
