# k_orient_brief grid-size probe (ORBX_DEBUG_OBDIV); profiling only
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
for v in ${DIVS:-1 2 4}; do
  ORBX_DEBUG_OBDIV=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --batch 64 --no-cpu-baseline > gpurun_out/probe/ob$v.json 2> gpurun_out/probe/ob$v.err || exit $?
  python -c "import json;d=json.load(open('gpurun_out/probe/ob$v.json'));print('div $v', d['value'], d['stages_ms_per_step'])"
done
