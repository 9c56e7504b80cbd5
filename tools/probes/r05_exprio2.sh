# pyramid + FAST issue priority on plans with a pyramid (base) vs off (ep0):
# extraction parity, then pipelined A/B per workload (3 pairs)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05ep bash tools/gpu_tests.sh tests/test_gpu_parity.py tests/test_stereo.py tests/test_bench_cli.py || { tail -30 gpurun_out/gtests_r05ep.log; exit 1; }
tail -1 gpurun_out/gtests_r05ep.log
for wl in c4 c1 c2 c5; do
  WL=$wl BATCH=0 STEPS=20 VARS="ep0 base ep0 base ep0 base" bash tools/variant_probe.sh | cut -d' ' -f1,2 | sed "s/^/$wl /" || exit 1
done
