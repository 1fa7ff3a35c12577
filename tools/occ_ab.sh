mkdir -p gpurun_out/occ && export CULL_AB_SCENES=Synthetic100k,W4_Optional,Bunny8Lights
for rep in 1 2; do for v in occ1 occ0 occ2; do
  L=gp1_raytracer_2223_amd/lib/exp/librtx_hip_$v.so
  RTX_HIP_LIB=$L timeout -k 10 120 python tools/cull_ab.py 30 - cull= > gpurun_out/occ/ab_${v}_$rep.txt 2>&1 || exit 1
  RTX_HIP_LIB=$L timeout -k 10 120 python tools/share_probe.py Synthetic100k 1920 1080 > gpurun_out/occ/share_syn_${v}_$rep.txt 2>&1 || exit 1
  RTX_HIP_LIB=$L timeout -k 10 120 python tools/share_probe.py Bunny8Lights 3840 2160 > gpurun_out/occ/share_b8_${v}_$rep.txt 2>&1 || exit 1
done; done
