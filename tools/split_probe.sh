# pipelined headline vs --split (sub-batches of the extraction on their own streams)
#   WLS="c4 c1" SPLITS="1 2 4" bash tools/split_probe.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/split
for wl in ${WLS:-c4}; do
  for sp in ${SPLITS:-1 2}; do
    timeout -k 10 200 python bench.py --workload $wl --split ${sp%%:*} $( [ "$sp" != "${sp%%:*}" ] && echo --match-whole ) --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-latency > gpurun_out/split/b_${wl}.json 2> gpurun_out/split/b_${wl}.err || exit $?
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], 'split', sys.argv[3], d['value'], d['unit'], d['ms_per_step'])" gpurun_out/split/b_${wl}.json $wl $sp
  done
done
