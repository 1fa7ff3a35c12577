#!/bin/bash
# HBM traffic of the render kernels per configuration, for bench.py's roofline.traffic and
# multi_gpu_configs.hbm_per_rank (run on the GPU box).  Two PMC passes per configuration
# (FETCH_SIZE and WRITE_SIZE cannot share one: MI355X_MICROARCH.md), each hard-killed if the
# profiler stalls; the summary keys every record on the SHA-256 of the librtx_hip.so used.
# Usage: bash tools/pmc_configs.sh <out name under gpurun_out> ["scene W H step;..."]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
NAME=${1:-pmc_configs}
OUT=gpurun_out/$NAME
mkdir -p $OUT
CONFIGS=${2:-"W4_Bunny 1920 1080 1;W4_Bunny 1920 1080 2;W4_Bunny 1920 1080 4;W4_Bunny 1920 1080 8;W4_Optional 1920 1080 1;Synthetic100k 1920 1080 1;Synthetic100k 1920 1080 2;Synthetic100k 1920 1080 4;Synthetic100k 1920 1080 8;Bunny8Lights 3840 2160 1;Bunny8Lights 3840 2160 2;Bunny8Lights 3840 2160 4;Bunny8Lights 3840 2160 8"}
FRAMES=${FRAMES:-40}
IFS=';' read -ra CFG <<< "$CONFIGS"
for c in "${CFG[@]}"; do
  read -r scene w h step <<< "$c"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    d=$OUT/${scene}_${w}x${h}_s${step}_$ctr
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d $d -o run --output-format csv -- python3 tools/pmc_driver.py $scene $w $h $step $FRAMES > $d.log 2>&1 || { echo "pmc pass $scene $w $h $step $ctr failed: stopping"; tail -5 $d.log; exit 1; }
  done
  echo "pmc ok: $c"
done
python3 tools/pmc_configs.py $OUT > $OUT/pmc_configs.json && echo "summary: $OUT/pmc_configs.json"
