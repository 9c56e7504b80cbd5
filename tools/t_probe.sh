# matcher list length probe: parity of variants (matcher tests), timing, resolver stats
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in t4 t6; do
  ORBX_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py -k "bow or match" > gpurun_out/tp_$v.log 2>&1 || exit $?
  tail -1 gpurun_out/tp_$v.log
done
VARS="base t4 t6 base t4" bash tools/variant_probe.sh || exit $?
ORBX_VARIANT=t4s timeout -k 10 120 python bench.py --steps 1 --warmup 0 --batch 64 --no-cpu-baseline > gpurun_out/t4s.txt 2>&1 || exit $?
grep "^RS" gpurun_out/t4s.txt | head -6
