# round-4 GPU session script: split-phase key sharing and part count A/B (tools/, not product)
mkdir -p gpurun_out/r04_sh
for L in share0 product; do
  if [ $L = product ]; then unset RTX_HIP_LIB; else export RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_$L.so; fi
  timeout -k 10 150 python -u tools/share_probe.py Synthetic100k 1920 1080 p64=RTX_SPLIT_PARTS:64 p256=RTX_SPLIT_PARTS:256 > gpurun_out/r04_sh/share_$L.log 2>&1
  CULL_AB_SCENES=W4_Optional,Synthetic100k timeout -k 10 120 python -u tools/cull_ab.py 50 - cull= p64=RTX_SPLIT_PARTS:64 p256=RTX_SPLIT_PARTS:256 > gpurun_out/r04_sh/ab_$L.log 2>&1
  echo "== $L"; cut -c1-400 gpurun_out/r04_sh/share_$L.log; cut -c1-330 gpurun_out/r04_sh/ab_$L.log
done
