# k_match_finalize register path: matcher parity, drop-in latency + kernel
# stats, serial/pipelined c4 and c1 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05fin bash tools/gpu_tests.sh tests/test_gpu_parity.py tests/test_cpp_adapter.py tests/test_bench_cli.py -k "bow or match or resolve or kf_frame or compat or adapter or bench" || { tail -30 gpurun_out/gtests_r05fin.log; exit 1; }
tail -1 gpurun_out/gtests_r05fin.log
timeout -k 10 120 python tools/bow_latency_probe.py 200 || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/bowlat3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/bow_latency_probe.py 60 > $OUT/log 2>&1 || exit 1
mkdir -p gpurun_out/probe
for wl in c4 c1; do
  timeout -k 10 180 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-latency > gpurun_out/probe/fin_$wl.json 2> gpurun_out/probe/fin_$wl.err || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], d['serial']['ms_per_step'], d['stages_ms_per_step']['match_finalize'])" gpurun_out/probe/fin_$wl.json $wl
done
