set -o pipefail
cd $GRAFT_REPO_ROOT
for wl in c2 c4 c1 c5; do
VARS="pk1 t30 f32 f64 f160 pk1 t30 f64" EXTRA_ARGS=--serial WL=$wl STEPS=20 bash tools/variant_probe.sh || exit $?
done
