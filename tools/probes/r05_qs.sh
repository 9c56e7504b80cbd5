set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c2 c4; do
VARS="prof qs1 qp0 prof qs1 qp0" EXTRA_ARGS=--serial WL=$wl STEPS=10 bash tools/variant_probe.sh || exit $?
done
