set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --batch 64 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/bench1.err; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --batch 64 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof1.log
