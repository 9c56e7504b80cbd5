# occupancy probes: extraction kernels with extra LDS per workgroup leave room
# for the matcher's kernels in the pipelined step (c4, batch 256)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
VARS="prof prof:ORBX_DEBUG_LDSPAD=2048,0,0 prof:ORBX_DEBUG_LDSPAD=0,3072,0 prof:ORBX_DEBUG_LDSPAD=0,0,5120 prof:ORBX_DEBUG_LDSPAD=2048,3072,5120 prof" \
  BATCH=256 WL=c4 STEPS=20 bash tools/variant_probe.sh
