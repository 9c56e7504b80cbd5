set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05g bash tools/gpu_tests.sh tests || { tail -40 gpurun_out/gtests_r05g.log; exit 1; }
tail -2 gpurun_out/gtests_r05g.log
R=r05g bash tools/round_final.sh || exit $?
