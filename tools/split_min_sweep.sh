#!/bin/bash
# The split threshold's cost floor (RTX_SPLIT_MIN_US, kSplitMinUs): serialized frame time of full frames and
# stripe shares for several floors (tools/share_once.py, warmed up).  Usage: bash tools/split_min_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for m in ${FLOORS:-0 30 60 100}; do
  for cfg in "W4_Optional 1920 1080 1" "W4_Optional 1920 1080 8" "Bunny8Lights 3840 2160 8" "W4_Bunny 1920 1080 8" \
             "Synthetic100k 1920 1080 1" "Synthetic100k 1920 1080 8" "Bunny8Lights 3840 2160 1"; do
    echo -n "floor $m us: "
    RTX_SPLIT_MIN_US=$m timeout -k 10 60 python tools/share_once.py $cfg 300 || exit $?
  done
done
