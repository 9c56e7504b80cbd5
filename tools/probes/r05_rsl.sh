# long-list rescan parity (release build), then the same cases under the
# RS_STATS build to count the rescans they trigger
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05rsl bash tools/gpu_tests.sh tests/test_gpu_parity.py -k "rescan_long_lists or heavy_contention or chunk_edges" || { tail -30 gpurun_out/gtests_r05rsl.log; exit 1; }
tail -1 gpurun_out/gtests_r05rsl.log
ORBX_VARIANT=rst timeout -k 10 300 python -u -m pytest -x -q -s -m gpu -p no:cacheprovider tests/test_gpu_parity.py -k "rescan_long_lists" > gpurun_out/rsl_stats.log 2>&1 || { tail -20 gpurun_out/rsl_stats.log; exit 1; }
grep "^RS unit" gpurun_out/rsl_stats.log | sed "s/^\.//" | awk "{h+=\$15; n++} END {print \"units\", n, \"rescans\", h}"
