set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05pf bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "extract or pyr or brief" || { tail -30 gpurun_out/gtests_r05pf.log; exit 1; }
tail -1 gpurun_out/gtests_r05pf.log
for wl in c4 c1 c5; do
VARS="pf1 pf0 pf1 pf0" EXTRA_ARGS=--serial WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
