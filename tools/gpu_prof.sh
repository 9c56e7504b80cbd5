# trace + traffic (FETCH/WRITE) + SQ counter passes for one tag; each GPU step bounded
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-run}
bash tools/profile.sh $TAG || exit $?
bash tools/pmc_sq.sh $TAG || exit $?
