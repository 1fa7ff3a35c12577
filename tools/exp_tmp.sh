cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
LIBS="${LIBS:-v11 oct}" ROUNDS=${ROUNDS:-3} SCENES=${SCENES:-W4_Bunny,W3,W4_Optional,Bunny8Lights,Synthetic100k} timeout -k 10 900 bash tools/ab.sh > gpurun_out/ab.log 2>&1; rc=$?
cat gpurun_out/ab.log
exit $rc
