#!/usr/bin/env python3
"""Summarise tools/pmc_configs.sh passes into the records bench.py reads
(profiles/r*/pmc_configs.json).  Per configuration: HBM bytes per launch of the main render
kernel (PHASE 0) and per frame (every render launch of the frame: PHASE 0 + the split
phases), 2 x FETCH_SIZE + WRITE_SIZE with FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950
tallies 128-B reads at 64 B).  The first two frames (identity order, first cost-ordered
frame) are dropped.

    python3 tools/pmc_configs.py <gpurun_out/pmc_configs dir>"""
import collections
import csv
import glob
import hashlib
import json
import os
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SKIP_FRAMES = 2


def per_dispatch(run_dir):
    """{dispatch id: (kernel name, value)} of one single-counter pass."""
    out = {}
    for f in glob.glob(f"{run_dir}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not k.startswith("void rtx_render_kernel<false"):
                continue
            did = int(r.get("Dispatch_Id") or r["Correlation_Id"])
            name, v = out.get(did, (k, 0.0))
            out[did] = (k, v + float(r["Counter_Value"]))   # summed over XCD / instance rows
    return out


def frames(disp):
    """Dispatches grouped per frame (ordered by id; a PHASE-0 launch closes its frame, the
    split phases of a frame are enqueued before it)."""
    groups, cur = [], []
    for did in sorted(disp):
        name, v = disp[did]
        cur.append((name, v))
        if name.startswith("void rtx_render_kernel<false, 0"):
            groups.append(cur)
            cur = []
    return groups[SKIP_FRAMES:]


def main():
    d = Path(sys.argv[1])
    lib = ROOT / "gp1_raytracer_2223_amd" / "lib" / "librtx_hip.so"
    lib_hash = hashlib.sha256(lib.read_bytes()).hexdigest()
    recs = []
    for fetch_dir in sorted(glob.glob(f"{d}/*_FETCH_SIZE")):
        base = fetch_dir[: -len("_FETCH_SIZE")]
        m = re.match(r"(.+)_(\d+)x(\d+)_s(\d+)$", os.path.basename(base))
        scene, W, H, step = m.group(1), int(m.group(2)), int(m.group(3)), int(m.group(4))
        fr = frames(per_dispatch(fetch_dir))
        wr = frames(per_dispatch(base + "_WRITE_SIZE"))
        if not fr or not wr:
            continue
        main_f = [sum(v for n, v in g if n.startswith("void rtx_render_kernel<false, 0")) for g in fr]
        main_w = [sum(v for n, v in g if n.startswith("void rtx_render_kernel<false, 0")) for g in wr]
        all_f = [sum(v for _, v in g) for g in fr]
        all_w = [sum(v for _, v in g) for g in wr]
        mean = lambda xs: sum(xs) / len(xs)  # noqa: E731
        kb = 1024.0
        # per phase (main kernel, split phases 1-3): HBM bytes per frame and their ratio to the
        # phase's algorithmic bytes = what it must write (uint32 frame 4 B/px for the main kernel
        # and PHASE 3, the 8-B hit key per heavy pixel for PHASE 1, the 4-B occlusion word for
        # PHASE 2) plus one read of the scene image
        phases = {}
        state = {}
        log = Path(base + "_FETCH_SIZE.log")
        if log.exists():
            for line in log.read_text().splitlines():
                if line.startswith("STATE "):
                    state = {k: int(v) for k, v in (kv.split("=") for kv in line.split()[1:])}
        rows = H if step == 1 else 16 * ((H // 16 + step - 1) // step)
        px = W * rows
        hp = 64 * state.get("heavy_tiles", 0)
        out_bytes = {0: 4 * max(0, px - hp), 1: 8 * hp, 2: 4 * hp, 3: 4 * hp}
        for ph in range(4):
            tag = f"void rtx_render_kernel<false, {ph}"
            pf = [sum(v for n, v in g if n.startswith(tag)) for g in fr]
            pw = [sum(v for n, v in g if n.startswith(tag)) for g in wr]
            nl = mean([sum(1 for n, _ in g if n.startswith(tag)) for g in fr])
            if nl == 0:
                continue
            b = int(round((2 * mean(pf) + mean(pw)) * kb))
            alg = out_bytes[ph] + state.get("scene_bytes", 0)
            phases[["main", "p1", "p2", "p3"][ph]] = {
                "hbm_bytes_per_frame": b, "launches_per_frame": round(nl, 2),
                "algorithmic_bytes": alg if state else None,
                "ratio_to_algorithmic": round(b / alg, 2) if state and alg else None}
        recs.append({
            "config": {"scene": scene, "width": W, "height": H, "views": 1, "stripe_step": step},
            "stripes": "rank 0's 16-row stripes" if step > 1 else "whole frame",
            "frames": len(fr),
            "fetch_kb_per_launch": round(mean(main_f), 1), "write_kb_per_launch": round(mean(main_w), 1),
            "hbm_bytes_per_launch": int(round((2 * mean(main_f) + mean(main_w)) * kb)),
            "hbm_bytes_per_frame": int(round((2 * mean(all_f) + mean(all_w)) * kb)),
            "split_launches_per_frame": round(mean([len(g) - 1 for g in fr]), 2),
            "phases": phases, "state": state,
            "lib_sha256": lib_hash,
        })
    print(json.dumps({"command": "bash tools/pmc_configs.sh (rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE, one pass each, "
                                 "-- python3 tools/pmc_driver.py <scene> <W> <H> <stripe_step> <frames>)",
                      "hbm_note": "bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (counters in KB); FETCH_SIZE doubled "
                                  "per MI355X_MICROARCH.md; Infinity-Cache hits are counted in FETCH_SIZE",
                      "records": recs}, indent=1))


if __name__ == "__main__":
    main()
