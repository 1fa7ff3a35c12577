# The animated loop with the device Update (rtx_anim_*) on the GPU box: the anim's own
# high-priority stream, its own stream at normal priority, and the context's stream (default).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/abd && cd gpurun_out/abd || exit 1
EXE=../../gp1_raytracer_2223_amd/lib/rtx_render
for cfg in "W4_Optional 1920 1080" "W4_Bunny 1920 1080"; do
  for f in 2 3; do
    for mode in high normal same; do
      echo "== $cfg inflight $f device-update ($mode)"
      case $mode in
        high) RTX_ANIM_OWN_STREAM=1 timeout -k 10 60 $EXE $cfg --benchmark 3 --inflight $f --device-update --out /tmp/anim.bmp --assets ../../gp1_raytracer_2223_amd/assets | grep -E "AVG" || exit 1 ;;
        normal) RTX_ANIM_OWN_STREAM=1 RTX_ANIM_STREAM_PRIO=normal timeout -k 10 60 $EXE $cfg --benchmark 3 --inflight $f --device-update --out /tmp/anim.bmp --assets ../../gp1_raytracer_2223_amd/assets | grep -E "AVG" || exit 1 ;;
        same) timeout -k 10 60 $EXE $cfg --benchmark 3 --inflight $f --device-update --out /tmp/anim.bmp --assets ../../gp1_raytracer_2223_amd/assets | grep -E "AVG" || exit 1 ;;
      esac
    done
  done
done
