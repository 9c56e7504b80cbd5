# (historical: RS_PRIO was removed after this A/B)
# resolver wave priority (s_setprio) in the pipelined step: base (0) vs 1 / 3
set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1 c2 c5; do
  WL=$wl BATCH=0 STEPS=20 VARS="base rp3 rp1 base rp3 rp1" bash tools/variant_probe.sh | cut -d' ' -f1,2 | sed "s/^/$wl /" || exit 1
done
