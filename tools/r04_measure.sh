#!/bin/bash
# Round-4 measurement set on the GPU box (results under gpurun_out/r04_meas, copied into
# profiles/r04 by hand): PMC traffic records of this build, then the driver's bench command,
# the default bench, and the rocprofv3 kernel trace of the driver's command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_meas
mkdir -p $OUT
timeout -k 10 400 bash tools/pmc_configs.sh r04_pmc > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
mkdir -p profiles/r04 && cp gpurun_out/r04_pmc/pmc_configs.json profiles/r04/pmc_configs.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { echo "bench driver failed"; tail -5 $OUT/bench_driver.err; exit 1; }
timeout -k 10 400 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench default failed"; tail -5 $OUT/bench_default.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
python3 - <<'PY'
import json
for n in ("bench_driver", "bench_default"):
    d = json.loads([l for l in open(f"gpurun_out/r04_meas/{n}.json") if l.startswith("{")][-1])
    r = d["roofline"]
    print(n, d["value"], d["ms_per_step"], "kernel_ms", r["kernel_ms"], "frac", r["frac"], "traffic", r["traffic"],
          "cpu", d["cpu_baseline"]["value"] if d.get("cpu_baseline") else None, "speedup", d.get("speedup_vs_cpu"))
PY
