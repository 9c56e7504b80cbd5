set -o pipefail
cd $GRAFT_REPO_ROOT
for v in prev "" prev ""; do
  ORBX_VARIANT=$v timeout -k 10 120 python bench.py --workload c5 --steps 10 --warmup 2 --batch 64 --no-cpu-baseline > gpurun_out/c5_$v.json 2>gpurun_out/c5_$v.err || exit $?
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print('c5', sys.argv[2], d['value'], d.get('stages_ms_per_step'))" gpurun_out/c5_$v.json "v=$v"
done
