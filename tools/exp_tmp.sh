cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
RTX_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err; rc=$?
echo "rc=$rc"; cat gpurun_out/bench_n2.json; tail -3 gpurun_out/bench_n2.err
RTX_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --steps 50 --warmup 5 > gpurun_out/bench_n4.json 2> gpurun_out/bench_n4.err; rc=$?
echo "rc=$rc"; cat gpurun_out/bench_n4.json; tail -3 gpurun_out/bench_n4.err
