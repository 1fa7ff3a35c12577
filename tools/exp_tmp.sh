cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q -x 2>&1 | tail -2 || exit 1
cd gpurun_out && mkdir -p bm && cd bm
for sc in W4_Bunny W4_Optional Bunny8Lights; do
echo "== $sc"; timeout -k 10 60 ../../gp1_raytracer_2223_amd/lib/rtx_render $sc 1920 1080 --benchmark 3 | grep "AVG\|frames" || exit 1
done
