# kernel staging in every drop-in call that stages through pinned memory:
# full GPU suite, then the drop-in SearchByBoW latency
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05stg2 bash tools/gpu_tests.sh tests || { tail -30 gpurun_out/gtests_r05stg2.log; exit 1; }
tail -1 gpurun_out/gtests_r05stg2.log
timeout -k 10 120 python tools/bow_latency_probe.py 300 || exit 1
