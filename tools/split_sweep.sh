# Split-rendering threshold sweep (RTX_SPLIT_FACTOR) over the mesh configs: frame time per factor.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for sc in ${SCENES:-"Synthetic100k 1920 1080|W4_Optional 1920 1080|Bunny8Lights 3840 2160|W4_Reference 1920 1080"}; do :; done
IFS='|' read -ra SCS <<< "${SCENES:-Synthetic100k 1920 1080|W4_Optional 1920 1080|Bunny8Lights 3840 2160|W4_Reference 1920 1080}"
for sc in "${SCS[@]}"; do
  for f in ${FACTORS:-1.25 1.5 1.75 2}; do
    RTX_SPLIT_FACTOR=$f timeout -k 10 120 python tools/split_probe.py $sc | sed "s/^/factor $f: /" || exit 1
  done
done
