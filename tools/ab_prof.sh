#!/bin/bash
# In-step A/B of one kernel: rocprofv3 kernel stats of bench.py with the in-tree library and with
# tools/_abl/liblgnn_<tag>.so, twice each; prints each run's average duration of kernels matching
# PATTERN and the step time. Usage (GPU box): PATTERN=k_s3_fbwd bash tools/ab_prof.sh <tag> [bench args]
set -uo pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/abprof
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do for v in intree $TAG; do
  if [ $v = intree ]; then LP=""; else LP=$GRAFT_REPO_ROOT/tools/_abl/liblgnn_$v.so; fi
  (cd /tmp && LGNN_LIB_PATH=$LP timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/${v}_$rep" -o t -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 20 \
    --cpu-seconds 0 --no-kernel-timing "$@" > "$OUT/${v}_$rep.json" 2> "$OUT/${v}_$rep.err") \
    || { tail -5 "$OUT/${v}_$rep.err"; exit 1; }
  python3 - "$OUT/${v}_$rep" "$v" "${PATTERN:-k_s3_fbwd}" "$OUT/${v}_$rep.json" <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if sys.argv[3] in r["Name"]]
d = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
print(sys.argv[2], [(r["Name"][:40], round(float(r["AverageNs"]) / 1e3, 2)) for r in rows], d["ms_per_step"])
PY
done; done
