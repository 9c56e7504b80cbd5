# extraction issue priority 3 (ep3) vs 2 (base), pipelined, 3 pairs
set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1 c5; do
  WL=$wl BATCH=0 STEPS=20 VARS="base ep3 base ep3 base ep3" bash tools/variant_probe.sh | cut -d' ' -f1,2 | sed "s/^/$wl /" || exit 1
done
