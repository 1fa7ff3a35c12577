#!/bin/bash
# Per-dispatch PMC counters of the device Update kernels (rtx_anim_build / rtx_anim_out), one
# rocprofv3 pass per counter group, over tools/anim_probe.py.  Usage: [LIB=anim7] bash tools/anim_pmc.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/anim_pmc
mkdir -p $OUT
[ -n "$LIB" ] && export RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_$LIB.so
i=0
IFS='|' read -ra GRPS <<< "${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM|SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY|SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY}"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/g$i -o run --output-format csv -- python3 tools/anim_probe.py W4_Optional > $OUT/g$i.log 2>&1 || { echo "group $i failed"; tail -5 $OUT/g$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys
for kname in ("rtx_anim_build", "rtx_anim_out"):
    agg = collections.defaultdict(list)
    for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    print(kname, "per dispatch:", "  ".join(f"{k} {v:.0f}" for k, v in sorted(m.items())))
PY
