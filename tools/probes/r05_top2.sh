# (historical: the MC_TOP3=2 variant was removed after this A/B)
# matcher candidates: per-lane top-2 (top2) vs top-3 (base) before the wave
# insertions -- serial-loop candidate times, then pipelined c4 / c1
set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1 c2 c5; do
  WL=$wl BATCH=0 STEPS=10 EXTRA_ARGS=--serial VARS="base top2 base top2" bash tools/variant_probe.sh | python3 -c "
import sys,ast
for ln in sys.stdin:
    t,v,rest=ln.split(' ',2); d=ast.literal_eval(rest.strip()); print('$wl', t, 'cand', d.get('match_candidates'))" || exit 1
done
for wl in c4 c1; do
  WL=$wl BATCH=0 STEPS=20 VARS="base top2 base top2" bash tools/variant_probe.sh | cut -d' ' -f1,2 || exit 1
done
