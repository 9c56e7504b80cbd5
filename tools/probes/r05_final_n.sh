# round-5 evidence after the drop-in kernel staging: full GPU suite, smoke,
# then kernel stats / traffic / SQ / bench lines per workload (round_final)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r05n bash tools/gpu_tests.sh tests || { tail -40 gpurun_out/gtests_r05n.log; exit 1; }
tail -2 gpurun_out/gtests_r05n.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
R=r05n bash tools/round_final.sh || exit $?
