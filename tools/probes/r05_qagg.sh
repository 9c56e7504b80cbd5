# (historical: the variant this measured was reverted)
# quadtree child / node counts aggregated per wave (QT_AGG_MAXS: base 64,
# qa0 = off, qa256, qa4k = every pass): extraction parity, serial-loop
# stage times per workload, the drop-in extraction latency
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05qa bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "extract or batched or plan or brief or quadtree or scale or threshold" || { tail -30 gpurun_out/gtests_r05qa.log; exit 1; }
tail -1 gpurun_out/gtests_r05qa.log
for wl in c4 c1 c2 c5; do
  WL=$wl BATCH=0 STEPS=10 EXTRA_ARGS=--serial VARS="qa0 base qa256 qa4k qa0 base" bash tools/variant_probe.sh | python3 -c "
import sys,ast
for ln in sys.stdin:
    t,v,rest=ln.split(' ',2); d=ast.literal_eval(rest.strip()); print(t, v, 'quadtree', d.get('quadtree'))" || exit 1
done
for v in qa0 base qa4k; do
  vv=""; [ $v != base ] && vv=$v
  echo -n "$v "; ORBX_VARIANT=$vv timeout -k 10 120 python tools/extract_latency_probe.py 200 || exit 1
done
