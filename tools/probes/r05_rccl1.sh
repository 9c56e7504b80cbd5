set -o pipefail
cd $GRAFT_REPO_ROOT
for v in "1 extract" "1 match" "1 own" "0 extract" "1 match" "1 own"; do
set -- $v
ORBX_BENCH_RCCL1=$1 timeout -k 10 300 python bench.py --workload c4 --steps 20 --warmup 5 --no-cpu-baseline --no-latency --xch-stream $2 > gpurun_out/rccl_c4.json 2> gpurun_out/rccl_c4.err || { tail -20 gpurun_out/rccl_c4.err; exit 1; }
python3 -c "import json,sys;L=open(sys.argv[1]).read().splitlines();assert len(L)==1,L[:3];d=json.loads(L[0]);print(sys.argv[2], d['value'], d['ms_per_step'], d['serial']['ms_per_step'], d['distributed']['backend'])" gpurun_out/rccl_c4.json "rccl$1-$2"
done
