# pyramid + FAST waves raised in issue arbitration (s_setprio, EX_PRIO 1 / 2)
# against the co-resident matcher in the pipelined step
set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1 c2 c5; do
  WL=$wl BATCH=0 STEPS=20 VARS="base ep2 ep1 base ep2 ep1" bash tools/variant_probe.sh | cut -d' ' -f1,2 | sed "s/^/$wl /" || exit 1
done
