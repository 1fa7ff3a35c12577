# round-4 GPU session script: parity suite, pair-kernel A/B, timelines (tools/, not product)
mkdir -p gpurun_out/r04_pair
RTX_PAIR=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r04_pair/tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04_pair/tests.log
[ $rc -ne 0 ] && { grep -n "FAILED\|Error\|assert" gpurun_out/r04_pair/tests.log | head -20; exit 1; }
export CULL_AB_SCENES=W4_Bunny,Bunny8Lights,Synthetic100k,W4_Optional
timeout -k 10 200 python -u tools/cull_ab.py 100 - cull= pair=RTX_PAIR:1 > gpurun_out/r04_pair/ab.log 2>&1
cut -c1-330 gpurun_out/r04_pair/ab.log
RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_pw8.so CULL_AB_SCENES=W4_Bunny,Bunny8Lights timeout -k 10 100 python -u tools/cull_ab.py 100 - pair=RTX_PAIR:1 > gpurun_out/r04_pair/ab_pw8.log 2>&1
cut -c1-200 gpurun_out/r04_pair/ab_pw8.log
export RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_stampslean.so
unset CULL_AB_SCENES
timeout -k 10 60 python -u tools/stamps.py Synthetic100k 1920 1080 > gpurun_out/r04_pair/st_syn.txt 2>&1
STAMPS_STRIPE=16,0,8 timeout -k 10 60 python -u tools/stamps.py Synthetic100k 1920 1080 > gpurun_out/r04_pair/st_syn_s8.txt 2>&1
timeout -k 10 60 python -u tools/stamps.py Bunny8Lights 3840 2160 > gpurun_out/r04_pair/st_b8.txt 2>&1
STAMPS_STRIPE=16,0,8 timeout -k 10 60 python -u tools/stamps.py Bunny8Lights 3840 2160 > gpurun_out/r04_pair/st_b8_s8.txt 2>&1
head -8 gpurun_out/r04_pair/st_*.txt
