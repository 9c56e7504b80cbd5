# build a profiling variant of liborbx.so with -D overrides:
#   bash tools/variant.sh NAME "-DPYR_U=2"   -> orb-slam-system_amd/liborbx_NAME.so
# select it at run time with ORBX_VARIANT=NAME (profiling only); variants
# are built with -DORBX_PROFILING, which enables the ORBX_DEBUG_* / ORBX_CHUNK
# environment knobs (a release liborbx.so never reads them)
set -e
cd "$(dirname "$0")/.."
make -s -j8 -C orb-slam-system_amd BUILD=build_$1 LIB=liborbx_$1.so EXTRA="-DORBX_PROFILING $2"
