# stage times with kernel phases cut short (ORBX_DEBUG_STOP); profiling only
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
for v in ${VARIANTS:-0 1 2 3 4 11}; do
  ORBX_DEBUG_STOP=$v timeout -k 10 120 python bench.py --steps 10 --warmup 2 --batch 64 --no-cpu-baseline > gpurun_out/probe/v$v.json 2> gpurun_out/probe/v$v.err || exit $?
done
