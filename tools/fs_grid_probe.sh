# k_fast_strips time vs persistent grid size (ORBX_DEBUG_FS_GRID); profiling only
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fsg
for k in ${GRIDS:-0 4 8 16}; do
  ORBX_DEBUG_FS_GRID=$k timeout -k 10 120 python bench.py --steps 10 --warmup 2 --batch 64 --no-cpu-baseline > gpurun_out/fsg/g$k.json 2> gpurun_out/fsg/g$k.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/fsg/g$k.json'));print('grid $k', d['value'], d['stages_ms_per_step']['fast_cells'])"
done
