# (historical probe) the candidates' waves at issue priority 2 (mcp2, a
# profiling build) vs none (base), pipelined c2 / c4
set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c2 c4; do
  WL=$wl BATCH=0 STEPS=20 VARS="base mcp2 base mcp2 base mcp2" bash tools/variant_probe.sh | cut -d' ' -f1,2 | sed "s/^/$wl /" || exit 1
done
