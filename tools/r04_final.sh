#!/bin/bash
# Final round-4 GPU pass: the GPU test suite, then tools/r04_measure.sh (PMC, benches, trace), then
# the headline-only kernel trace.  Results under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_meas
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_meas/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -20 gpurun_out/r04_meas/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r04_meas/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> gpurun_out/r04_meas/gpu_tests.log 2>&1 || { echo "smoke failed"; exit 1; }
bash tools/r04_measure.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_meas/trace_head -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/r04_meas/trace_head.log 2>&1 || { echo "headline trace failed"; exit 1; }
