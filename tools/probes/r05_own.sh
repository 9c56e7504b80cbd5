set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05own bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "extract or overflow or plan" || { tail -30 gpurun_out/gtests_r05own.log; exit 1; }
tail -1 gpurun_out/gtests_r05own.log
for wl in c4 c2 c1; do
VARS="own noown own noown" EXTRA_ARGS=--serial WL=$wl STEPS=10 bash tools/variant_probe.sh || exit $?
done
