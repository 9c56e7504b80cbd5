set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c4 c1 c5; do
VARS="prof prof:ORBX_DEBUG_PYR_TILE=2 prof:ORBX_DEBUG_PYR_TILE=3 prof:ORBX_DEBUG_PYR_TILE=4 prof:ORBX_DEBUG_PYR_TILE=5 prof" EXTRA_ARGS=--serial WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
