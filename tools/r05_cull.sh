#!/bin/bash
# Round 5, the segment-tree cull records on the GPU box: the cull tests, a kernel trace of the
# moving-camera loop (the record kernels' durations), the moving-camera loop itself and the
# W4_Optional F6 loop with and without the cull.  Usage: bash tools/r05_cull.sh [tag]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_cull}
mkdir -p $OUT
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_cull.py -x -v --timeout 120 --timeout-method thread \
  > $OUT/pytest_cull.log 2>&1 || { echo "cull tests failed"; tail -30 $OUT/pytest_cull.log; exit 1; }
tail -2 $OUT/pytest_cull.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- \
  python3 tools/moving_camera.py 100 Synthetic100k,W4_Optional > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
timeout -k 10 200 python3 tools/moving_camera.py 400 > $OUT/moving_camera.txt 2>&1 || { echo "moving camera failed"; tail -20 $OUT/moving_camera.txt; exit 1; }
cat $OUT/moving_camera.txt
EXE=gp1_raytracer_2223_amd/lib/rtx_render
for f in 1 3 1 3; do
  for c in cull no_cull; do
    echo "== W4_Optional 1920x1080 inflight $f $c" >> $OUT/anim.txt
    if [ $c = no_cull ]; then export RTX_NO_CULL=1; else unset RTX_NO_CULL; fi
    timeout -k 10 60 $EXE W4_Optional 1920 1080 --benchmark 3 --inflight $f --out /tmp/anim.bmp \
      --assets gp1_raytracer_2223_amd/assets >> $OUT/anim.txt 2>&1 || { echo "anim failed"; tail -20 $OUT/anim.txt; exit 1; }
  done
done
unset RTX_NO_CULL
grep -E "==|AVG" $OUT/anim.txt
