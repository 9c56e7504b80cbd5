# single-frame (drop-in orbx_extract, 1080p) kernel durations per profiling
# variant: VARS="pf qs1 qp0 qp2" bash tools/qt_latency_probe.sh TAG
# -> gpurun_out/qtlat_TAG/<var>/run_kernel_stats.csv, summary in summary.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/qtlat_${1:-run}
mkdir -p $OUT
for v in ${VARS:-pf}; do
  name=${v%%:*}; envs=""
  [ "$v" != "$name" ] && envs=${v#*:}
  mkdir -p $OUT/$v
  env ORBX_VARIANT=$name $envs timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o run -- python3 tools/extract_latency_probe.py 60 > $OUT/$v/log 2>&1 || exit 1
  python3 - "$OUT/$v" "$v" >> $OUT/summary.txt <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
out = []
for r in rows:
    n = r["Name"].split("(")[0].split("::")[-1]
    if n.startswith("k_"):
        out.append("%s %.1fus" % (n, float(r["AverageNs"]) / 1e3))
lat = open(sys.argv[1] + "/log").read().strip().splitlines()
print(sys.argv[2], "|", " ".join(out), "|", [l for l in lat if l.startswith("p50")][:1])
PY
done
cat $OUT/summary.txt
