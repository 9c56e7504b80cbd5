set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05st bash tools/gpu_tests.sh tests/test_stereo.py || { tail -30 gpurun_out/gtests_r05st.log; exit 1; }
tail -1 gpurun_out/gtests_r05st.log
VARS="kp2 kp1 kp2 kp1" EXTRA_ARGS=--serial WL=c5 STEPS=20 bash tools/variant_probe.sh || exit $?
VARS="kp2 kp1" WL=c5 STEPS=20 bash tools/variant_probe.sh || exit $?
