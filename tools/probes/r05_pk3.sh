set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1 c2; do
VARS="pk1 w6 rt2 pk1 w6" EXTRA_ARGS=--serial WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
