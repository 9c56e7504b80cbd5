# drop-in SearchByBoW latency: plain timing, then a kernel + copy trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python tools/bow_latency_probe.py 200 || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/bowlat
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT -o run -- python3 tools/bow_latency_probe.py 60 > $OUT/log 2>&1 || exit 1
ls $OUT
