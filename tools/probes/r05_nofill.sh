# pipelined window without fill / drain (step k = batch k-1's matching +
# batch k's extraction): bench CLI tests (incl. the 2-rank pipelined
# equality), then c4/c1/c2/c5 at the driver's 20 / 5 and c4 at 80 steps, and
# the one-rank RCCL rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05nf bash tools/gpu_tests.sh tests/test_bench_cli.py tests/test_multirank_gpu.py || { tail -30 gpurun_out/gtests_r05nf.log; exit 1; }
tail -1 gpurun_out/gtests_r05nf.log
mkdir -p gpurun_out/probe
run() {  # tag wl args...
  t=$1; wl=$2; shift 2
  timeout -k 10 180 python bench.py --workload $wl --no-cpu-baseline --no-latency "$@" > gpurun_out/probe/nf_$t.json 2> gpurun_out/probe/nf_$t.err || { tail -5 gpurun_out/probe/nf_$t.err; return 1; }
  python3 -c "import json,sys;L=open(sys.argv[1]).read().splitlines();assert len(L)==1;d=json.loads(L[0]);print(sys.argv[2], d['value'], d['ms_per_step'], 'drain', d.get('pipeline_drain_ms'), 'serial', d['serial']['ms_per_step'], d['distributed']['backend'])" gpurun_out/probe/nf_$t.json "$t"
}
for wl in c4 c1 c2 c5; do run ${wl}_20 $wl --steps 20 --warmup 5 || exit 1; done
run c4_80 c4 --steps 80 --warmup 5 || exit 1
run c4_5 c4 --steps 5 --warmup 5 || exit 1
ORBX_BENCH_RCCL1=1 run c4_rccl1 c4 --steps 20 --warmup 5 || exit 1
run c4_20b c4 --steps 20 --warmup 5 || exit 1
