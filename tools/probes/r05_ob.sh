set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05ob bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "extract or brief or sincos" || exit $?
tail -1 gpurun_out/gtests_r05ob.log
for wl in c4 c1 c2; do
VARS="oldob prof oldrint oldob prof oldrint" EXTRA_ARGS=--serial WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
