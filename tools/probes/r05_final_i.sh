set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05i bash tools/gpu_tests.sh tests || { tail -40 gpurun_out/gtests_r05i.log; exit 1; }
tail -2 gpurun_out/gtests_r05i.log
R=r05i bash tools/round_final.sh || exit $?
