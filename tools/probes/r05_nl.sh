set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05nl bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "bow or match_plan" || { tail -30 gpurun_out/gtests_r05nl.log; exit 1; }
tail -1 gpurun_out/gtests_r05nl.log
for wl in c4 c1 c2; do
VARS="cur lds cur lds" WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
