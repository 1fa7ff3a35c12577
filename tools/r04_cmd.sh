# round-4 GPU session script: parity of the fused split launch, and its A/B (tools/, not product)
mkdir -p gpurun_out/r04_fu
timeout -k 10 300 python -u -m pytest tests/test_gpu_cull.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r04_fu/tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04_fu/tests.log
[ $rc -ne 0 ] && { grep -n "FAILED\|Error\|assert" gpurun_out/r04_fu/tests.log | head -20; exit 1; }
CULL_AB_SCENES=W4_Optional,Synthetic100k,Bunny8Lights timeout -k 10 150 python -u tools/cull_ab.py 50 - cull= unfused=RTX_SPLIT_FUSED:0 > gpurun_out/r04_fu/ab.log 2>&1
cut -c1-330 gpurun_out/r04_fu/ab.log
timeout -k 10 200 python -u tools/share_probe.py Synthetic100k 1920 1080 unfused=RTX_SPLIT_FUSED:0 > gpurun_out/r04_fu/share_syn.log 2>&1
cut -c1-400 gpurun_out/r04_fu/share_syn.log
timeout -k 10 200 python -u tools/share_probe.py Bunny8Lights 3840 2160 unfused=RTX_SPLIT_FUSED:0 > gpurun_out/r04_fu/share_b8.log 2>&1
cut -c1-400 gpurun_out/r04_fu/share_b8.log
