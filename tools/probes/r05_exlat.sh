# drop-in extraction latency: plain timing, then a kernel + copy trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python tools/extract_latency_probe.py 200 || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/exlat
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT -o run -- python3 tools/extract_latency_probe.py 40 > $OUT/log 2>&1 || exit 1
