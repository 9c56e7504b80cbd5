set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05mf bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "extract or brief" || { tail -30 gpurun_out/gtests_r05mf.log; exit 1; }
tail -1 gpurun_out/gtests_r05mf.log
for wl in c4 c1 c2; do
VARS="h0 mf1 mf3 mf9 h0" EXTRA_ARGS=--serial WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
