mkdir -p gpurun_out/r04_st
timeout -k 10 240 python -u -m pytest tests/test_gpu_deep_bvh.py tests/test_gpu_cull.py tests/test_gpu_configs.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r04_st/tests.log 2>&1; tail -2 gpurun_out/r04_st/tests.log
export CULL_AB_SCENES=Synthetic100k,W4_Optional
for L in share0 share1 product; do
  if [ $L = product ]; then unset RTX_HIP_LIB; else export RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_$L.so; fi
  timeout -k 10 120 python -u tools/cull_ab.py 50 - cull= p64=RTX_SPLIT_PARTS:64 > gpurun_out/r04_st/ab_$L.log 2>&1
  echo "== $L"; cut -c1-300 gpurun_out/r04_st/ab_$L.log
done
export RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_stampslean.so
timeout -k 10 90 python -u tools/stamps.py Synthetic100k 1920 1080 > gpurun_out/r04_st/syn_split.txt 2>&1
RTX_SPLIT=0 timeout -k 10 90 python -u tools/stamps.py Synthetic100k 1920 1080 > gpurun_out/r04_st/syn_nosplit.txt 2>&1
cat gpurun_out/r04_st/syn_split.txt gpurun_out/r04_st/syn_nosplit.txt
STAMPS_STRIPE=16,0,8 timeout -k 10 90 python -u tools/stamps.py Synthetic100k 1920 1080 > gpurun_out/r04_st/syn_s8.txt 2>&1
timeout -k 10 90 python -u tools/stamps.py Bunny8Lights 3840 2160 > gpurun_out/r04_st/b8_full.txt 2>&1
STAMPS_STRIPE=16,0,8 timeout -k 10 90 python -u tools/stamps.py Bunny8Lights 3840 2160 > gpurun_out/r04_st/b8_s8.txt 2>&1
head -12 gpurun_out/r04_st/syn_s8.txt gpurun_out/r04_st/b8_full.txt gpurun_out/r04_st/b8_s8.txt
