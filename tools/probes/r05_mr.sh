set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05mr bash tools/gpu_tests.sh tests/test_multirank_gpu.py || { tail -40 gpurun_out/gtests_r05mr.log; exit 1; }
grep -E "PASS|FAIL|SKIP" gpurun_out/gtests_r05mr.log | tail -6
