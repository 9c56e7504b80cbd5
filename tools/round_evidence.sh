# round-end evidence on the GPU box: profiles (trace + traffic + SQ), then the
# default bench line (with the CPU baseline) using the fresh traffic summary
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
bash tools/gpu_prof.sh $TAG || exit $?
timeout -k 10 600 python bench.py --traffic gpurun_out/prof_$TAG/traffic.json > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
