#!/bin/bash
# Instruction counts per wave of the render kernel for several experiment builds
# (tools/build_variant.py), one rocprofv3 PMC pass each.  Usage: LIBS="cur abl_SMESH" bash tools/pmc_variants.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcv
mkdir -p $OUT
for L in $LIBS; do
  RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_$L.so timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH \
    -d $OUT/$L -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$L.log 2>&1 || { echo "$L failed"; tail -5 $OUT/$L.log; exit 1; }
  python3 - "$OUT/$L" "$L" <<'PY'
import csv, collections, glob, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("void rtx_render_kernel<false, 0>"):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in agg.items()}
w = m.get("SQ_WAVES", 1)
print(f"{sys.argv[2]:12s} waves {w:8.0f}  VALU {m.get('SQ_INSTS_VALU',0)/w:7.1f}  SALU {m.get('SQ_INSTS_SALU',0)/w:7.1f}  BRANCH {m.get('SQ_INSTS_BRANCH',0)/w:6.1f} per wave")
PY
done
