set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05g1 bash tools/gpu_tests.sh tests || { tail -40 gpurun_out/gtests_r05g1.log; exit 1; }
tail -2 gpurun_out/gtests_r05g1.log
timeout -k 10 300 python bench.py --workload c4 > gpurun_out/r05g1_bench_c4.json 2> gpurun_out/r05g1_bench_c4.err || exit $?
head -c 600 gpurun_out/r05g1_bench_c4.json
