# k_pyramid time vs last-level tile size (ORBX_DEBUG_PYR_TILE); profiling only
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pyr
for k in ${TILES:-0 1 2 3 4}; do
  ORBX_DEBUG_PYR_TILE=$k timeout -k 10 120 python bench.py --steps 10 --warmup 2 --batch 64 --no-cpu-baseline > gpurun_out/pyr/t$k.json 2> gpurun_out/pyr/t$k.err || exit $?
done
