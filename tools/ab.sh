#!/bin/bash
# A/B timing of experiment builds (tools/build_variant.py) in alternating rounds on one GPU box.
# Usage: LIBS="prev new" [AB=ablate|cull|share] [SCENES=W4_Bunny,W3] [ROUNDS=2] bash tools/ab.sh
#   AB=ablate (default)  tools/ablate.py: kernel ms per scene and mode
#   AB=cull              tools/cull_ab.py: kernel ms per config, bit-identity to the unculled walk
#   AB=share             tools/share_probe.py Synthetic100k 1080p: one-GPU strong-scaling shares
# (round 4's occ_ab.sh was AB=cull then AB=share over LIBS="occ1 occ0 occ2")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in $LIBS; do
    echo "== $L (round $r)"
    export RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_$L.so
    case ${AB:-ablate} in
      ablate) ABLATE_MODES=${MODES:-combined+shadows} ABLATE_SCENES=${SCENES:-W4_Bunny,W3,W4_Optional,Bunny8Lights} \
                timeout -k 10 300 python tools/ablate.py ${ITERS:-50} || exit $? ;;
      cull)   CULL_AB_SCENES=${SCENES:-Synthetic100k,W4_Optional,Bunny8Lights} \
                timeout -k 10 300 python tools/cull_ab.py ${ITERS:-30} - cull= > gpurun_out/ab/cull_${L}_$r.txt 2>&1 || exit $?
              cat gpurun_out/ab/cull_${L}_$r.txt ;;
      share)  timeout -k 10 300 python tools/share_probe.py Synthetic100k 1920 1080 > gpurun_out/ab/share_${L}_$r.txt 2>&1 || exit $?
              cat gpurun_out/ab/share_${L}_$r.txt ;;
    esac
  done
done
