cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x 2>&1 | tail -3 || exit 1
for lib in gp1_raytracer_2223_amd/lib/librtx_hip.so gp1_raytracer_2223_amd/lib/exp/librtx_hip_prev.so gp1_raytracer_2223_amd/lib/librtx_hip.so gp1_raytracer_2223_amd/lib/exp/librtx_hip_prev.so; do
echo "== $lib"
RTX_HIP_LIB=$lib ABLATE_SCENES=W4_Bunny,W3,Bunny8Lights,W4_Optional ABLATE_MODES=combined+shadows timeout -k 10 200 python tools/ablate.py 30 || exit 1
done
