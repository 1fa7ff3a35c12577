#!/bin/bash
# Split-rendering phase durations per split factor (rocprofv3 kernel trace of tools/split_probe.py):
# the main kernel beside the P1 -> P2 -> P3 chain.  Usage: bash tools/split_phases.sh <scene> "<factors>"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/split_phases_$1
mkdir -p $OUT
for f in $2; do
  RTX_SPLIT_FACTOR=$f timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/t$f -o run --output-format csv -- \
    python3 tools/split_probe.py $1 1920 1080 > $OUT/log$f.txt 2>&1 || { tail -5 $OUT/log$f.txt; exit 1; }
  echo "== factor $f: $(grep heavy $OUT/log$f.txt)"
  python3 tools/kstats.py $(find $OUT/t$f -name "*kernel_trace.csv") rtx_render_kernel
done
