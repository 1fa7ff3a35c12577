#!/bin/bash
# Headline A/B: alternate bench.py runs (the driver's command, headline only) over experiment builds
# on one GPU box.  Usage: LIBS="r05 r06a" [ROUNDS=3] [STEPS=20] [WARMUP=5] bash tools/ab_bench.sh
# One JSON summary line per run: lib, round, value, ms_per_step, kernel_ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for r in $(seq 1 ${ROUNDS:-3}); do
  for L in $LIBS; do
    RTX_HIP_LIB=gp1_raytracer_2223_amd/lib/exp/librtx_hip_$L.so timeout -k 10 120 \
      python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} --no-extra --no-cpu-baseline --no-gather \
      > gpurun_out/ab/bench_${L}_$r.json 2> gpurun_out/ab/bench_${L}_$r.err || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps({'lib': sys.argv[2], 'round': int(sys.argv[3]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms']}))" gpurun_out/ab/bench_${L}_$r.json $L $r
  done
done
