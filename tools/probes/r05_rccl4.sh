set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05mr2 bash tools/gpu_tests.sh tests/test_multirank_gpu.py tests/test_bench_cli.py || { tail -40 gpurun_out/gtests_r05mr2.log; exit 1; }
tail -1 gpurun_out/gtests_r05mr2.log
for wl in c4 c5; do
for r in 0 1; do
ORBX_BENCH_RCCL1=$r timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 5 --no-cpu-baseline --no-latency > gpurun_out/rccl_$wl.json 2> gpurun_out/rccl_$wl.err || { tail -20 gpurun_out/rccl_$wl.err; exit 1; }
python3 -c "import json,sys;L=open(sys.argv[1]).read().splitlines();assert len(L)==1;d=json.loads(L[0]);print(sys.argv[2], d['value'], d['ms_per_step'], d['serial']['ms_per_step'], d['distributed']['backend'])" gpurun_out/rccl_$wl.json "$wl-rccl$r"
done
done
ORBX_BENCH_SHARE_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --workload c1 --batch 64 --steps 5 --warmup 2 --no-cpu-baseline --no-latency > gpurun_out/share2.json 2> gpurun_out/share2.err || { tail -20 gpurun_out/share2.err; exit 1; }
python3 -c "import json,sys;L=open(sys.argv[1]).read().splitlines();d=json.loads(L[-1]);print('share2', len(L), d['value'], d['n_gpus'], d['distributed']['backend'], d['distributed']['world_size'])" gpurun_out/share2.json
