# round-4 GPU session script: wave priority of the split launches, A/B (tools/, not product)
mkdir -p gpurun_out/r04_pr
for L in prio0 prio1 prio3; do
  export RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_$L.so
  CULL_AB_SCENES=W4_Optional,Synthetic100k timeout -k 10 150 python -u tools/cull_ab.py 50 - cull= > gpurun_out/r04_pr/ab_$L.log 2>&1
  timeout -k 10 200 python -u tools/share_probe.py Synthetic100k 1920 1080 > gpurun_out/r04_pr/share_$L.log 2>&1
  echo "== $L"; cut -c1-200 gpurun_out/r04_pr/ab_$L.log; cut -c1-400 gpurun_out/r04_pr/share_$L.log
done
