# (historical probe) stereo matcher waves at issue priority 2 (smp2,
# profiling build) vs none (base), pipelined c5
set -o pipefail
cd $GRAFT_REPO_ROOT
WL=c5 BATCH=0 STEPS=20 VARS="base smp2 base smp2 base smp2" bash tools/variant_probe.sh | cut -d' ' -f1,2 || exit 1
