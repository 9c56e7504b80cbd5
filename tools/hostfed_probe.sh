# host-fed leg vs the number of H2D copy streams (ORBX_BENCH_H2D_STREAMS)
#   NS="1 2 4" bash tools/hostfed_probe.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
for n in ${NS:-1 2 4}; do
  ORBX_BENCH_H2D_STREAMS=$n timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/probe/hf_$n.json 2> gpurun_out/probe/hf_$n.err || exit $?
  python -c "import json,sys;d=json.load(open(sys.argv[1]))['host_fed'];print('streams', sys.argv[2], d['value'], d['pcie_h2d_gbs'], d['counts_equal_resident_run'])" gpurun_out/probe/hf_$n.json $n
done
