cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x 2>&1 | tail -3 || exit 1
for sc in Synthetic100k W4_Optional W4_Bunny Bunny8Lights W4_Reference W3; do timeout -k 10 100 python tools/split_probe.py $sc || exit 1; done
