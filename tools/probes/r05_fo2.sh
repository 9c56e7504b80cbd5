set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c1 c4 c5; do
VARS="old n6 f2 cc old n6 f2 cc" EXTRA_ARGS=--serial WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
