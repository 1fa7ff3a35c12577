#!/bin/bash
# Round-5 measurement set (results under gpurun_out/, copied into profiles/r05 by hand): the
# end-of-round pass (tools/final_pass.sh: PMC records incl. per-phase bytes, driver's and default
# bench lines, kernel traces), the record kernels alone, the moving-camera loop, the split tuner.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/final_pass.sh r05 --no-tests || exit 1
OUT=gpurun_out/r05_meas
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/rec_trace -o run --output-format csv -- python3 tools/cull_record_probe.py 20 > $OUT/rec.log 2>&1 || { echo "record probe failed"; exit 1; }
python3 tools/kstats.py $(find $OUT/rec_trace -name "*kernel_trace.csv") cull,sched > $OUT/record_kernels_isolated.txt
timeout -k 10 300 python3 tools/moving_camera.py 400 > $OUT/moving_camera_inflight2.txt 2>&1 || { echo "moving camera failed"; exit 1; }
MC_INFLIGHT=1 timeout -k 10 300 python3 tools/moving_camera.py 300 > $OUT/moving_camera_serial.txt 2>&1 || { echo "moving camera serial failed"; exit 1; }
timeout -k 10 300 python3 tools/split_tune_probe.py Synthetic100k,W4_Optional 1.5,2 > $OUT/split_tune_probe.txt 2>&1 || { echo "tune probe failed"; exit 1; }
cat $OUT/record_kernels_isolated.txt
