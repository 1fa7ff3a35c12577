cd $GRAFT_REPO_ROOT
E=gp1_raytracer_2223_amd/lib/exp
for lib in $E/librtx_hip_prev.so $E/librtx_hip_vmem.so $E/librtx_hip_prev.so $E/librtx_hip_vmem.so; do
echo "== $lib"
RTX_HIP_LIB=$lib ABLATE_SCENES=W4_Bunny,W4_Optional,Synthetic100k ABLATE_MODES=combined+shadows timeout -k 10 250 python tools/ablate.py 10 || exit 1
done
