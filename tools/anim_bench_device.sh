cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/abd && cd gpurun_out/abd || exit 1
EXE=../../gp1_raytracer_2223_amd/lib/rtx_render
for cfg in "W4_Optional 1920 1080" "W4_Bunny 1920 1080"; do
  for f in 1 2 3; do
    echo "== $cfg inflight $f device-update (own stream)"
    timeout -k 10 60 $EXE $cfg --benchmark 3 --inflight $f --device-update --out /tmp/anim.bmp --assets ../../gp1_raytracer_2223_amd/assets | grep -E "AVG|per frame" || exit 1
    echo "== $cfg inflight $f device-update (context stream)"
    RTX_ANIM_SAME_STREAM=1 timeout -k 10 60 $EXE $cfg --benchmark 3 --inflight $f --device-update --out /tmp/anim.bmp --assets ../../gp1_raytracer_2223_amd/assets | grep -E "AVG|per frame" || exit 1
  done
done
