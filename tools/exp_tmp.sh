cd $GRAFT_REPO_ROOT
for o in 1 0; do
echo "== RTX_TILE_ORDER=$o"
RTX_TILE_ORDER=$o ABLATE_SCENES=W4_Bunny,W3,Bunny8Lights,W4_Optional,Synthetic100k ABLATE_MODES=combined+shadows timeout -k 10 200 python tools/ablate.py 30 || exit 1
RTX_TILE_ORDER=$o RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_stamps.so timeout -k 10 120 python tools/stamps.py Bunny8Lights 3840 2160 | head -12
done
