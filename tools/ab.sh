#!/bin/bash
# A/B kernel timing of experiment builds (tools/build_variant.py) in alternating rounds on
# one GPU box.  Usage: LIBS="prev new" [SCENES=W4_Bunny,W3] [ROUNDS=2] bash tools/ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in $LIBS; do
    echo "== $L (round $r)"
    RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_$L.so ABLATE_MODES=${MODES:-combined+shadows} \
      ABLATE_SCENES=${SCENES:-W4_Bunny,W3,W4_Optional,Bunny8Lights} timeout -k 10 300 python tools/ablate.py ${ITERS:-50} || exit $?
  done
done
