#!/bin/bash
# GPU-box check: parity tests, then a short bench.  Stops at the first abnormal exit
# (fault/abort/timeout), continues past ordinary test failures (exit 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc"
tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench exit $rc"
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $rc
