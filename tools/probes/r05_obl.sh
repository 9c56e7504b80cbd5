set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1 c2; do
VARS="prof obl prof obl" EXTRA_ARGS=--serial WL=$wl STEPS=10 bash tools/variant_probe.sh || exit $?
done
