# (historical: the variant this measured was reverted)
# k_quadtree_few for small launches (drop-in extraction): full GPU suite,
# the extraction latency probe + trace, and the c4 line's latency leg
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05qf bash tools/gpu_tests.sh tests || { tail -30 gpurun_out/gtests_r05qf.log; exit 1; }
tail -1 gpurun_out/gtests_r05qf.log
timeout -k 10 120 python tools/extract_latency_probe.py 200 || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/exlat2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/extract_latency_probe.py 40 > $OUT/log 2>&1 || exit 1
mkdir -p gpurun_out/probe
timeout -k 10 300 python bench.py --workload c4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/probe/qf_c4.json 2> gpurun_out/probe/qf_c4.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/probe/qf_c4.json'));L=d['latency']
print(d['value'], d['ms_per_step'], L['extract_1920x1080']['p50_us'], L['extract_1920x1080']['p99_us'], L['extract_640x480']['p50_us'], L['compat_operator_1920x1080']['operator_with_mvImagePyramid']['p50_us'], L['search_by_bow_2000x2000']['p50_us'])"
