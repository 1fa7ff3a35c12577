cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x 2>&1 | tail -2 || exit 1
E=gp1_raytracer_2223_amd/lib/exp
for lib in $E/librtx_hip_prev.so $E/librtx_hip_new.so $E/librtx_hip_prev.so $E/librtx_hip_new.so; do
echo "== $lib"
RTX_HIP_LIB=$lib ABLATE_SCENES=W4_Bunny,W3,W4_Optional,Bunny8Lights,Synthetic100k ABLATE_MODES=combined+shadows timeout -k 10 250 python tools/ablate.py 20 || exit 1
done
