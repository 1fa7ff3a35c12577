#!/bin/bash
# Per-pixel instruction counts of the W4_Bunny render kernel, one-packet vs the round-4 pair kernel
# (RTX_PAIR; the kernel is in git history, commit 38d4bf8, removed after this A/B: DESIGN.md §9).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_pair
mkdir -p $OUT
for P in 0 1; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH" "SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
    i=$((i+1))
    RTX_PAIR=$P timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/p$P/g$i -o run --output-format csv -- python3 tools/pmc_driver.py W4_Bunny 1920 1080 1 40 > $OUT/p$P.g$i.log 2>&1 || { echo "pair=$P group $i failed"; tail -5 $OUT/p$P.g$i.log; exit 1; }
  done
  python3 - "$OUT/p$P" "$P" <<'PY'
import csv, collections, glob, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if n.startswith("void rtx_render_pair_kernel") or n.startswith("void rtx_render_kernel<false, 0, false, 3570"):
            agg[(n[:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
m = collections.defaultdict(dict)
for (n, c), v in agg.items():
    m[n][c] = sum(v) / len(v)
for n, d in m.items():
    px = 1920 * 1080 / 64.0
    print(f"pair={sys.argv[2]} {n}: " + "  ".join(f"{k} {v / px:.1f}" for k, v in sorted(d.items())) + "  (per 64 pixels)")
PY
done
