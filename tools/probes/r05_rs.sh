# resolve walk: look-ahead waits fixed, rescans batched (RS_RU) -- matcher
# parity, then same-run A/B of the committed kernel (rsold) vs base (RS_RU=8), RS_RU=4/16
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05rs bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "bow or match or resolve or kf_frame" || { tail -30 gpurun_out/gtests_r05rs.log; exit 1; }
tail -1 gpurun_out/gtests_r05rs.log; grep -c PASSED gpurun_out/gtests_r05rs.log
for wl in c4 c1 c2 c5; do
  WL=$wl BATCH=0 STEPS=10 EXTRA_ARGS=--serial VARS="rsold base rsru4 rsru16 rsold base" bash tools/variant_probe.sh || exit 1
done
