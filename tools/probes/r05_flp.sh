# (historical: FS_LOADPRIO was removed after this A/B)
# FAST waves one priority level higher until their strip loads are issued
# (flp) vs the shipped constant priority (base), pipelined + serial FAST
set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1 c5; do
  WL=$wl BATCH=0 STEPS=20 VARS="base flp base flp base flp" bash tools/variant_probe.sh | cut -d' ' -f1,2 | sed "s/^/$wl /" || exit 1
done
WL=c4 BATCH=0 STEPS=10 EXTRA_ARGS=--serial VARS="base flp base flp" bash tools/variant_probe.sh | python3 -c "
import sys,ast
for ln in sys.stdin:
    t,v,rest=ln.split(' ',2); d=ast.literal_eval(rest.strip()); print('serial', t, d.get('fast_cells'))"
