cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/anim_pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SMEM -d gpurun_out/anim_pmc/p1 -o run --output-format csv -- python3 tools/anim_probe.py W4_Optional 640 360 > gpurun_out/anim_pmc/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY -d gpurun_out/anim_pmc/p2 -o run --output-format csv -- python3 tools/anim_probe.py W4_Optional 640 360 > gpurun_out/anim_pmc/p2.log 2>&1 || exit 2
find gpurun_out/anim_pmc -name "*counter_collection.csv"
