# column-split candidate kernel for launches with few workgroups: matcher
# parity, then the drop-in SearchByBoW latency and a c4 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05cs bash tools/gpu_tests.sh tests/test_gpu_parity.py tests/test_projection.py tests/test_cpp_adapter.py -k "bow or match or resolve or kf_frame or compat or adapter" || { tail -30 gpurun_out/gtests_r05cs.log; exit 1; }
tail -1 gpurun_out/gtests_r05cs.log
timeout -k 10 120 python tools/bow_latency_probe.py 200 || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/bowlat2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/bow_latency_probe.py 60 > $OUT/log 2>&1 || exit 1
