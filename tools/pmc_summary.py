"""Summarise a tools/profile.sh output dir: mean counter value per dispatch of the render kernel.

Usage: python tools/pmc_summary.py <prof dir> [version tag]
With a version tag the output is the full record bench.py reads (profiles/r01/pmc_summary.json):
config of the default bench command, HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) KB."""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
out = {}
meta = {}
for f in sorted(glob.glob(f"{d}/pmc*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if k.startswith(("void rtx_render_kernel<false, 0>", "void rtx_render_kernel<false, 0, false")):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
                                      "SGPR_Count")}
    for k, v in agg.items():
        out[k] = round(sum(v) / len(v), 1)
w = out.get("SQ_WAVES", 1)
derived = {}
for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM_RD"):
    if k in out:
        derived[k + "_per_wave"] = round(out[k] / w, 1)
if "SQ_THREAD_CYCLES_VALU" in out and "SQ_ACTIVE_INST_VALU" in out:
    derived["valu_lane_utilisation"] = round(out["SQ_THREAD_CYCLES_VALU"] / (64 * out["SQ_ACTIVE_INST_VALU"]), 3)
if "SQ_WAIT_ANY" in out and "SQ_WAVE_CYCLES" in out:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        derived[k + "_frac_of_wave_cycles"] = round(out[k] / out["SQ_WAVE_CYCLES"], 3)
rec = {"counters": out, "derived": derived, "dispatch": meta}
if len(sys.argv) > 2:
    rec = {"kernel": "rtx_render_kernel<false, 0>",
           "config": {"scene": "W4_Bunny", "width": 1920, "height": 1080, "views": 1},
           "command": "rocprofv3 --pmc <group> -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline "
                      "(tools/profile.sh, one group per pass)",
           **rec,
           "hbm_bytes_per_launch": int(round((2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024)),
           "hbm_note": "2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes); FETCH_SIZE doubled per MI355X_MICROARCH.md "
                       "(gfx950 tallies 128-B reads at 64 B). WRITE_SIZE = 4 B/pixel frame store.",
           "kernel_version": sys.argv[2] + " (profiles/r01/ablate_history.md)"}
print(json.dumps(rec, indent=1))
