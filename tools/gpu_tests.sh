# GPU test subset on the box: python -u pytest with per-test timeout; args = pytest selectors
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-t}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider "$@" > gpurun_out/gtests_$TAG.log 2>&1
rc=$?; echo "EXIT $rc" >> gpurun_out/gtests_$TAG.log; exit $rc
