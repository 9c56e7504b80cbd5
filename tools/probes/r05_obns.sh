# BRIEF upper bound: the per-keypoint output stores never issued (obns),
# serial-loop stage times (orient_brief) against the release build
set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1 c2; do
  WL=$wl BATCH=0 STEPS=10 EXTRA_ARGS=--serial VARS="base obns base obns" bash tools/variant_probe.sh || exit 1
done
