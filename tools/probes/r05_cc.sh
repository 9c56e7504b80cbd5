set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/ovf_probe.py || exit $?
TAG=r05cc bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "extract or overflow" || { tail -30 gpurun_out/gtests_r05cc.log; exit 1; }
tail -1 gpurun_out/gtests_r05cc.log
for wl in c1 c4 c5; do
VARS="base old base old" EXTRA_ARGS=--serial WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
