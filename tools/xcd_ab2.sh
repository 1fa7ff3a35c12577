#!/bin/bash
# XCD-affine dispatch with Latin-square block classes (RTX_XCD_BLOCKS builds): frame times with the re-deal
# on / off per build, then the main launch's L2 hit rate and fetch bytes for Synthetic100k.
# Usage: LIBS="xcd8 xcd16" bash tools/xcd_ab2.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r06/xcd2
mkdir -p $OUT
for L in $LIBS; do
  export RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_$L.so
  for x in 0 1; do
    for cfg in "Synthetic100k 1920 1080 1" "W4_Optional 1920 1080 1" "Bunny8Lights 3840 2160 1" "W4_Bunny 1920 1080 1"; do
      echo -n "$L xcd $x: "
      RTX_XCD_ORDER=$x timeout -k 10 60 python tools/share_once.py $cfg 300 || exit $?
    done
  done
  for ctr in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $ctr | cut -d' ' -f1)
    RTX_XCD_ORDER=1 RTX_SPLIT_FACTOR=2.3 timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/${L}_$tag -o run --output-format csv -- python3 tools/share_once.py Synthetic100k 1920 1080 1 40 > $OUT/${L}_$tag.log 2>&1 || { echo "pmc $L $ctr failed"; exit 1; }
  done
done
echo done
