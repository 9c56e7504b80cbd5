# GPU box: full -m gpu suite, then the default bench line (N=1), each bounded
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-t}
TAG=$TAG bash tools/gpu_tests.sh || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
