"""Per-kernel PMC means of a tools/profile.sh output dir: every render phase (PHASE 0 main
kernel, split phases 1-3) and the scheduler kernels, one line per kernel with the counters
per dispatch and per wave.  Usage: python tools/pmc_phases.py <prof dir> [out.json]"""
import collections
import csv
import glob
import json
import re
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{d}/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for name, cs in agg.items():
    m = {k: sum(v) / len(v) for k, v in cs.items()}
    w = m.get("SQ_WAVES", 0) or 1
    rec = {"per_dispatch": {k: round(v, 1) for k, v in m.items()},
           "per_wave": {k: round(v / w, 1) for k, v in m.items() if k.startswith("SQ_INSTS")}}
    if "SQ_WAVE_CYCLES" in m:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in m:
                rec.setdefault("frac_of_wave_cycles", {})[k] = round(m[k] / m["SQ_WAVE_CYCLES"], 3)
    if "SQ_ACTIVE_INST_VALU" in m and "GRBM_GUI_ACTIVE" in m:
        # VALU busy fraction of the SIMDs over the dispatch: each wave64 VALU instruction holds
        # a SIMD-32 for 2 cycles; 256 CUs x 4 SIMDs (MI355X_MICROARCH.md).  GRBM_GUI_ACTIVE is
        # summed over the 8 XCDs (Bunny 1080p: 1.6 M for a 74 us kernel at ~2.4 GHz).
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        rec["gpu_active_us"] = round(cyc / 2400.0, 1)
        if "SQ_INSTS_VALU" in m:
            rec["valu_issue_frac"] = round(2 * m["SQ_INSTS_VALU"] / (cyc * 1024), 3)
    out[name] = rec
    print(name, json.dumps(rec))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
