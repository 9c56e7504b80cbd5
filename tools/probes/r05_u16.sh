set -o pipefail
cd $GRAFT_REPO_ROOT
ORBX_VARIANT=u16a TAG=r05u16a bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "brief" || exit $?
tail -1 gpurun_out/gtests_r05u16a.log
for wl in c4 c1 c2; do
VARS="prof fold u16a u16l abit prof" EXTRA_ARGS=--serial WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
