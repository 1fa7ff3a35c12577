#!/bin/bash
# End-of-round GPU pass (results under gpurun_out/<round>_meas, copied into profiles/<round> by
# hand): the GPU test suite and smoke(), PMC traffic records of this build (tools/pmc_configs.sh),
# the driver's bench command, the default bench, and rocprofv3 kernel traces of the driver's
# command (whole line, then the headline only).  Usage: bash tools/final_pass.sh r05 [--no-tests]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${1:?round tag, e.g. r05}
OUT=gpurun_out/${R}_meas
mkdir -p $OUT profiles/$R
if [ "$2" != "--no-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -20 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" >> $OUT/gpu_tests.log 2>&1 || { echo "smoke failed"; exit 1; }
fi
timeout -k 10 600 bash tools/pmc_configs.sh ${R}_pmc > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
cp gpurun_out/${R}_pmc/pmc_configs.json profiles/$R/pmc_configs.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench driver failed"; tail -5 $OUT/bench_driver.err; exit 1; }
timeout -k 10 400 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench default failed"; tail -5 $OUT/bench_default.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_head -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-extra --no-cpu-baseline > $OUT/trace_head.log 2>&1 || { echo "headline trace failed"; exit 1; }
OUT=$OUT python3 - <<'PY'
import json, os
for n in ("bench_driver", "bench_default"):
    d = json.loads([l for l in open(f"{os.environ['OUT']}/{n}.json") if l.startswith("{")][-1])
    r = d["roofline"]
    print(n, d["value"], d["ms_per_step"], "kernel_ms", r["kernel_ms"], "frac", r["frac"], "traffic", r["traffic"],
          "cpu", d["cpu_baseline"]["value"] if d.get("cpu_baseline") else None, "speedup", d.get("speedup_vs_cpu"))
PY
