#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/ablate.py 50 > gpurun_out/ablate.txt 2>&1; rc=$?
cat gpurun_out/ablate.txt; exit $rc
