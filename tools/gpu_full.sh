#!/bin/bash
# GPU-box round check: the -m gpu suite, the default bench line, the PMC traffic records of
# this build, and a rocprofv3 kernel trace of the driver's bench command.  Every GPU step has
# its own time limit and the chain stops at the first abnormal exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-full}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -rf --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc"; tail -4 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
echo "bench ok"; head -c 600 $OUT/bench.json; echo
[ "${SKIP_PMC:-0}" = 1 ] || bash tools/pmc_configs.sh ${1:-full}_pmc || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
echo "trace ok"
find $OUT/trace -name "*kernel_stats.csv" -exec head -8 {} \;
