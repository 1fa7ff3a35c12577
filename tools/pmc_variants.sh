#!/bin/bash
# Per-wave PMC counts of the render kernel for several experiment builds
# (tools/build_variant.py), one rocprofv3 pass per (build, counter group).
# Usage: LIBS="cur abl_SMESH" [PMC_GROUPS="A B|C D"] [BENCH_ARGS=...] bash tools/pmc_variants.sh
# Default group: instruction counts.  Stops at the first failed pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcv
mkdir -p $OUT
IFS='|' read -ra GRPS <<< "${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH}"
for L in $LIBS; do
  export RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_$L.so
  i=0
  for grp in "${GRPS[@]}"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/$L/g$i -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --inflight 1 \
      --no-cpu-baseline --no-gather --no-extra ${BENCH_ARGS:-} > $OUT/$L.g$i.log 2>&1 || { echo "$L group $i failed"; tail -5 $OUT/$L.g$i.log; exit 1; }
  done
  python3 - "$OUT/$L" "$L" <<'PY'
import csv, collections, glob, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith(("void rtx_render_kernel<false, 0>", "void rtx_render_kernel<false, 0, false")):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in agg.items()}
w = m.get("SQ_WAVES", 32400.0)
print(f"{sys.argv[2]:12s} " + "  ".join(f"{k} {v / w:.2f}" for k, v in sorted(m.items()) if k != "SQ_WAVES") + "  (per wave)")
PY
done
