cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x 2>&1 | tail -3
ABLATE_SCENES=W4_Bunny,W3,Bunny8Lights,W4_Optional,Synthetic100k ABLATE_MODES=combined+shadows,combined timeout -k 10 200 python tools/ablate.py 30
