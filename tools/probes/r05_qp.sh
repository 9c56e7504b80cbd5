set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c2 c4; do
VARS="prof qp0 qp1 qp2 qp3 qp4 qp5 qp7 prof" EXTRA_ARGS=--serial WL=$wl STEPS=10 bash tools/variant_probe.sh || exit $?
done
