set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05fo bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "extract or overflow or brief or match_plan" || { tail -30 gpurun_out/gtests_r05fo.log; exit 1; }
tail -1 gpurun_out/gtests_r05fo.log
for wl in c4 c1 c2 c5; do
VARS="n7 old n6 n7 old" EXTRA_ARGS=--serial WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
