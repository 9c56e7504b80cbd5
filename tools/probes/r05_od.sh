# (historical: the variant this measured was reverted)
# drop-in SearchByBoW outputs written straight to the pinned buffer (base)
# vs the device arena + a copy back (od0)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05od bash tools/gpu_tests.sh tests/test_gpu_parity.py tests/test_cpp_adapter.py -k "bow or kf_frame or compat or adapter" || { tail -30 gpurun_out/gtests_r05od.log; exit 1; }
tail -1 gpurun_out/gtests_r05od.log
for r in 1 2 3; do
  for v in base od0; do
    vv=""; [ $v != base ] && vv=$v
    echo -n "$v "; ORBX_VARIANT=$vv timeout -k 10 120 python tools/bow_latency_probe.py 300 || exit 1
  done
done
