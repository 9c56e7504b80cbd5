# build liborbx_prev.so from a commit (default HEAD) for same-run A/B against
# the working tree: bash tools/prev_build.sh [commit]; then VARS="prev base"
set -e
cd "$(dirname "$0")/.."
C=${1:-HEAD}
rm -rf /tmp/orbx_prev_wt /tmp/orbx_prev_build
git worktree add -f /tmp/orbx_prev_wt "$C" -q
make -s -j8 -C /tmp/orbx_prev_wt/orb-slam-system_amd BUILD=/tmp/orbx_prev_build LIB=$PWD/orb-slam-system_amd/liborbx_prev.so
git worktree remove --force /tmp/orbx_prev_wt
