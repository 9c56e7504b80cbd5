# BRIEF outputs stored one keypoint late (OB_DEFER, base) vs at the end of
# their own iteration (obd0): extraction parity, then serial + pipelined A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05obd bash tools/gpu_tests.sh tests/test_gpu_parity.py || { tail -30 gpurun_out/gtests_r05obd.log; exit 1; }
tail -1 gpurun_out/gtests_r05obd.log; grep -c PASSED gpurun_out/gtests_r05obd.log
for wl in c4 c1 c2 c5; do
  WL=$wl BATCH=0 STEPS=10 EXTRA_ARGS=--serial VARS="obd0 base obd0 base" bash tools/variant_probe.sh || exit 1
done
for wl in c4 c1; do
  WL=$wl BATCH=0 STEPS=20 VARS="obd0 base obd0 base" bash tools/variant_probe.sh || exit 1
done
