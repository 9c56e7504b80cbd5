set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c2 c1 c4; do
VARS="prof qj12 qj20 qtg qtp prof" EXTRA_ARGS=--serial BATCH=0 WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
