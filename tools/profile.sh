#!/bin/bash
# rocprofv3 passes for the headline bench (run on the GPU box).
#   1) kernel trace + stats (durations)   2..n) one PMC group per pass
# Usage: [BENCH_ARGS="--scene X --width W --height H"] [PMC_GROUPS="A B|C D"] bash tools/profile.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd "$PWD" && export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="python3 bench.py --steps ${TRACE_STEPS:-100} --warmup 10 --no-cpu-baseline --inflight 1 ${BENCH_ARGS:-}"
set -o pipefail
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $BENCH > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/trace.log; exit 1; }
echo "trace ok"
i=0
PMCLIST=${PMC_GROUPS:-"FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM|SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS|GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH|SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA|SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU"}
IFS='|' read -ra GRPS <<< "$PMCLIST"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  # one counter group per pass, hard-killed if the profiler stalls; stop at the first failure
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py --steps ${PMC_STEPS:-20} --warmup 2 --no-cpu-baseline --inflight 1 ${BENCH_ARGS:-} > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($grp) failed: stopping"; tail -5 $OUT/pmc$i.log; exit 1; }
done
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
find $OUT -name "*.csv" | head -50
