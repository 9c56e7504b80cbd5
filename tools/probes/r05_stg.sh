# drop-in SearchByBoW: inputs staged by a kernel (base) vs a DMA copy (stg0)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05stg bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "bow or kf_frame" || { tail -30 gpurun_out/gtests_r05stg.log; exit 1; }
tail -1 gpurun_out/gtests_r05stg.log
for r in 1 2 3; do
  for v in base stg0; do
    vv=""; [ $v != base ] && vv=$v
    echo -n "$v "; ORBX_VARIANT=$vv timeout -k 10 120 python tools/bow_latency_probe.py 300 || exit 1
  done
done
