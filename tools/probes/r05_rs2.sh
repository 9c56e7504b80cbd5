# pipelined-step A/B of the rescan batch (resolve VGPRs 104 / 178 / RU=4)
set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1; do
  WL=$wl BATCH=0 STEPS=20 VARS="rsold base rsru4 rsold base rsru4" bash tools/variant_probe.sh || exit 1
done
