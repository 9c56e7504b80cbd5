# bench throughput vs frames per step (1 GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
for b in ${BATCHES:-32 64 128 256}; do
  timeout -k 10 240 python bench.py --steps 10 --warmup 2 --batch $b --no-cpu-baseline > gpurun_out/sweep/b$b.json 2> gpurun_out/sweep/b$b.err || exit $?
done
