"""Multi-rank partition (bench.py / DESIGN.md §6) on CPU with gloo, world_size 2 and 4:
each rank renders only its 16-row stripes of every view (oracle as the renderer, since
this container has no GPU); stitching the ranks' stripes must give the single-rank frame
bit for bit, each rank must get the same number of pixels, and no pixel is rendered twice.
The transport here (gather to rank 0) is test-only: bench.py moves no data between ranks."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _owned_rows(H, stripe, rank, world, view):
    first = (rank - view) % world
    return np.array([(y // stripe) % world == first for y in range(H)])


def _worker(rank, world, port, W, H, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests")]
    import torch
    import oracle_bind
    from gp1_raytracer_2223_amd import abi
    from gp1_raytracer_2223_amd.scene import HostScene
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hs = HostScene("W4_Bunny")
    s, cam = hs.view()
    views = bench.make_views(cam, world)
    frames = []
    count = 0
    for f in range(world):
        buf = np.zeros(W * H, np.uint32)
        # rtx_render_views semantics: view f owns stripes s % world == (rank - f) mod world
        p = abi.make_params(W, H, stripe_rows=16, stripe_first=(rank - f) % world, stripe_step=world)
        oracle_bind.render(s, views[f], p, threads=2, want_rgb=False, out_px=buf)
        count += int(_owned_rows(H, 16, rank, world, f).sum()) * W
        frames.append(torch.from_numpy(buf.view(np.int32)))
    gathered = [[torch.zeros(W * H, dtype=torch.int32) for _ in range(world)] for _ in range(world)]
    for f in range(world):
        dist.all_gather(gathered[f], frames[f])
    counts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(counts, torch.tensor([count]))
    if rank == 0:
        stitched = []
        for f in range(world):
            img = np.zeros(W * H, np.uint32)
            for r in range(world):
                rows = _owned_rows(H, 16, r, world, f)
                img.reshape(H, W)[rows] = gathered[f][r].numpy().view(np.uint32).reshape(H, W)[rows]
            ref, _ = oracle_bind.render(s, views[f], abi.make_params(W, H), threads=2, want_rgb=False)
            stitched.append(bool(np.array_equal(img, ref)))
        q.put((stitched, [int(c.item()) for c in counts]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_stripe_partition_gloo(world):
    W, H = 96, 96
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + world + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    stitched, counts = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(stitched), stitched
    assert sum(counts) == world * W * H          # every pixel of every view exactly once
    assert len(set(counts)) == 1                 # weak scaling: equal share per rank


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["views", "frame"])
def test_bench_two_ranks_hip_shmctl(mode, tmp_path):
    """The real multi-rank path on the HIP renderer: bench.py under torch.distributed.run
    with 2 ranks pinned to device 0 (RTX_BENCH_DEVICE; the driver's N-GPU runs map rank r
    to device r), coordinated by bench.py's shared-memory control block (ShmCtl: barriers and
    the max-over-ranks step time; no process group).  `views` (the default, weak scaling): 2 views per step, each
    striped over both ranks; `frame` (strong): one Bunny 1080p frame per step.  Each rank
    gathers its stripes into the shared page-locked host frames; rank 0 checks view 0 (the
    reference camera) against the reference's SHA-256 (bench.py `parity`)."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    world = 2
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, RTX_BENCH_DEVICE="0", MASTER_ADDR="127.0.0.1")
    port = 29700 + os.getpid() % 200 + (0 if mode == "views" else 1)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(root / "bench.py"), "--gpus", str(world),
           "--steps", "20", "--warmup", "5", "--no-cpu-baseline", "--mode", mode]
    out = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-4000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    r = json.loads(line)
    assert r["n_gpus"] == world and r["scaling"] == ("weak" if mode == "views" else "strong")
    assert r["parity"]["bit_exact"] is True, r["parity"]
    views = world if mode == "views" else 1
    assert r["roofline"]["frame_pixels_counted"] == views * 1920 * 1080   # every pixel exactly once
    assert r["host_gather"]["mpix_s"] > 0


def _ctl_worker(rank, world, port, q):
    import sys
    import time
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests")]
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_PORT=str(port))
    import bench
    d = bench.Dist()
    out = []
    for k in range(50):   # back-to-back reductions reuse the two value slots
        if rank == k % world:
            time.sleep(0.002)   # a late rank: nobody may leave the barrier before it arrives
        out.append((d.max(float(rank * 10 + k)), d.sum_i64([rank + 1, k])))
    g = d.gather([float(rank), 2.0 * rank])
    d.barrier()
    d.close()
    q.put((rank, out, g.tolist()))


@pytest.mark.parametrize("world", [2, 4])
def test_bench_control_plane_shm(world):
    """bench.py's control plane between rank processes (ShmCtl: barrier, max, sum, gather
    through one /dev/shm block, no torch in the bench process): every rank sees every
    reduction's result over all ranks, for 50 reductions in a row with a late rank each time."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31000 + world + os.getpid() % 1000
    procs = [ctx.Process(target=_ctl_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (o, g)) for r, o, g in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        out, g = res[r]
        for k, (mx, sm) in enumerate(out):
            assert mx == float((world - 1) * 10 + k)
            assert sm == [world * (world + 1) // 2, world * k]
        assert g == [[float(i), 2.0 * i] for i in range(world)]
    assert not [f for f in os.listdir("/dev/shm") if f.startswith(f"rtx_ctl_{port}_")]


@pytest.mark.gpu
def test_bench_one_gpu_contract(tmp_path):
    """The driver's N = 1 command (`bench.py --gpus 1 --steps 20 --warmup 5`, here with a 1-frame CPU
    sample): one JSON line with the contract's fields; `value` = pixels / ms_per_step; the roofline
    object; the CPU baseline and `speedup_vs_cpu` against its best configuration; every extra
    workload with its parity and the one-GPU strong-scaling predictor (efficiency = t_full / (s x the
    slowest share)); the culled lines' `frac` counts the work the culled walk executes, the
    reference-equivalent rate beside it."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    cmd = [sys.executable, str(root / "bench.py"), "--gpus", "1", "--steps", "20", "--warmup", "5", "--cpu-frames", "1"]
    out = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-4000:]
    r = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in r, k
    assert r["n_gpus"] == 1 and r["steps"] == 20 and r["warmup"] == 5 and r["higher_is_better"] is True
    assert abs(r["value"] - 1920 * 1080 / (r["ms_per_step"] * 1e-3) / 1e6) <= 1e-3 * r["value"]
    rf = r["roofline"]
    assert rf["bound"] in ("valu", "hbm", "mfma") and 0 < rf["frac"] < 1 and rf["peak"] > 0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    cpu = r["cpu_baseline"]
    assert cpu["kind"] in ("reference", "port") and cpu["value"] > 0 and cpu["cores"] >= 1
    assert cpu["value"] >= cpu["all_threads_mpix_s"] - 1e-6   # the best configuration measured
    assert abs(r["speedup_vs_cpu"] - r["value"] / cpu["value"]) <= 0.1 + 1e-3 * r["speedup_vs_cpu"]
    assert r["parity"]["bit_exact"] is True and r["parity_configs_all_ok"] is True
    scenes = {e["scene"]: e for e in r["multi_gpu_configs"]}
    for name, e in scenes.items():
        assert e["parity"]["ok"] is True, name
        sp = e["strong_scaling_predictor"]
        for s in (2, 4, 8):
            x = sp[f"s{s}"]
            assert len(x["share_ms"]) == s
            assert abs(x["efficiency"] - sp["t_full_ms"] / (s * max(x["share_ms"]))) < 1e-3
            y = sp["inflight"][f"s{s}"]   # the same with the bench's frames in flight
            assert len(y["share_ms"]) == s
            assert abs(y["efficiency"] - sp["inflight"]["t_full_ms"] / (s * max(y["share_ms"]))) < 1e-3
    assert "W4_Bunny" in scenes   # the headline scene's one-frame leg
    assert "flop_basis" in scenes["Synthetic100k"]["roofline_rank0"]
    assert "flop_basis" not in scenes["Bunny8Lights"]["roofline_rank0"]
    for name in ("Synthetic100k", "W4_Optional"):   # the culled scenes: `frac` is executed work
        rr = scenes[name]["roofline_rank0"]
        assert rr["flop_basis"].startswith("executed"), (name, rr)
        assert 0 < rr["frac"] < rr["frac_reference_equivalent"], (name, rr)
        assert abs(rr["frac"] - rr["achieved"] / rr["peak"]) < 1e-3
        assert abs(rr["frac_reference_equivalent"] - rr["achieved_reference_equivalent"] / rr["peak"]) < 1e-3
