# pyramid + FAST phase / bound probes (c4, batch 256, serial stage timers)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
VARS="samesrc nostore prof" EXTRA_ARGS=--serial BATCH=256 WL=c4 STEPS=10 bash tools/variant_probe.sh
