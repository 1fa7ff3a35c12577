#!/bin/bash
# Animated frame loop (the reference's F6 benchmark) on the GPU box: per scene, the serial
# loop (--inflight 1) beside the overlapped one (2, 3).  Usage: bash tools/anim_bench.sh [windows]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/anim && cd gpurun_out/anim || exit 1
EXE=../../gp1_raytracer_2223_amd/lib/rtx_render
for cfg in "W4_Optional 1920 1080" "W4_Bunny 1920 1080" "Bunny8Lights 3840 2160" "W4_Reference 1920 1080"; do
  for f in 1 2 3; do
    echo "== $cfg inflight $f"
    timeout -k 10 60 $EXE $cfg --benchmark ${1:-3} --inflight $f --out /tmp/anim.bmp --assets ../../gp1_raytracer_2223_amd/assets | grep -v "BENCHMARK\|wrote" || exit 1
  done
done
# the same loop with the Update on the device (rtx_anim_*)
for cfg in "W4_Optional 1920 1080" "W4_Bunny 1920 1080" "W4_Reference 1920 1080"; do
  for f in 1 3; do
    echo "== $cfg inflight $f device-update"
    timeout -k 10 60 $EXE $cfg --benchmark ${1:-3} --inflight $f --device-update --out /tmp/anim.bmp --assets ../../gp1_raytracer_2223_amd/assets | grep -v "BENCHMARK\|wrote" || exit 1
  done
done
