set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05grp bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "extract or overflow or brief or stereo" || { tail -30 gpurun_out/gtests_r05grp.log; exit 1; }
tail -1 gpurun_out/gtests_r05grp.log
for wl in c1 c5; do
VARS="grp prev grp prev" EXTRA_ARGS=--serial WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
