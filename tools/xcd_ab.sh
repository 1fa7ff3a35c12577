#!/bin/bash
# XCD-affine dispatch (RTX_XCD_ORDER=1) against the cost order alone: serialized frame times
# (tools/share_once.py, warmed up) and, per phase, the L2's memory-side fetch bytes and hit/miss counts
# (rocprofv3 --pmc, one counter group per pass).  Usage: bash tools/xcd_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06/xcd
mkdir -p $OUT
for r in 1 2; do
  for x in 0 1; do
    for cfg in "Synthetic100k 1920 1080 1" "W4_Optional 1920 1080 1" "Bunny8Lights 3840 2160 1" "W4_Bunny 1920 1080 1" \
               "Synthetic100k 1920 1080 8"; do
      echo -n "xcd $x round $r: "
      RTX_XCD_ORDER=$x timeout -k 10 60 python tools/share_once.py $cfg 300 || exit $?
    done
  done
done
for x in 0 1; do
  for ctr in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $ctr | cut -d' ' -f1)
    RTX_XCD_ORDER=$x RTX_SPLIT_FACTOR=2.3 timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/syn_x${x}_$tag -o run --output-format csv -- python3 tools/share_once.py Synthetic100k 1920 1080 1 40 > $OUT/syn_x${x}_$tag.log 2>&1 || { echo "pmc $x $ctr failed"; tail -5 $OUT/syn_x${x}_$tag.log; exit 1; }
  done
done
echo done
