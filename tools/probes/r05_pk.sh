set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05pk bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "bow or match_plan or descriptor" || { tail -30 gpurun_out/gtests_r05pk.log; exit 1; }
tail -1 gpurun_out/gtests_r05pk.log
for wl in c4 c1 c2; do
VARS="pk1 pk0 t30 pk1 pk0" EXTRA_ARGS=--serial WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
