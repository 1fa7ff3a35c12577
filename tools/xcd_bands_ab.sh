#!/bin/bash
# XCD bands (RTX_XCD_BANDS=1: band x of the image on XCD x) against the default dispatch, both
# in the experiment build:
# full-size parity of every config with bands on, kernel time A/B in alternating rounds, and
# FETCH_SIZE of Synthetic100k both ways (run on the GPU box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/xcd_bands
mkdir -p $OUT
# the experiment build (on the CPU beforehand): python tools/build_variant.py bands -DRTX_XCD_BANDS=1
export RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_bands.so
RTX_TEST_XCD_BANDS=1 RTX_XCD_BANDS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 300 \
  --timeout-method thread > $OUT/parity_bands.log 2>&1 || { tail -20 $OUT/parity_bands.log; exit 1; }
tail -2 $OUT/parity_bands.log
for r in 1 2; do
  for B in 0 1; do
    echo "== bands $B (round $r)"
    RTX_XCD_BANDS=$B ABLATE_MODES=combined+shadows ABLATE_SCENES=${SCENES:-Synthetic100k,W4_Bunny,Bunny8Lights,W4_Optional,W3} \
      timeout -k 10 300 python tools/ablate.py ${ITERS:-50} || exit $?
  done
done
for B in 0 1; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    d=$OUT/syn_b${B}_$ctr
    RTX_XCD_BANDS=$B timeout -s KILL 120 rocprofv3 --pmc $ctr -d $d -o run --output-format csv -- \
      python3 tools/pmc_driver.py Synthetic100k 1920 1080 1 40 > $d.log 2>&1 || { echo "pmc $B $ctr failed"; tail -5 $d.log; exit 1; }
  done
done
echo done
