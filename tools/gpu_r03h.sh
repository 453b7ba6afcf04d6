#!/bin/bash
# Round-3 (late) GPU session: the whole -m gpu suite, then an A/B of the in-tree library against
# tools/_abl/liblgnn_$AB.so on the C2 bench (per-step time and the dominant kernel's duration).
# Usage (GPU box, repo root): AB=base bash tools/gpu_r03h.sh <tag> [pytest selection...]
set -uo pipefail
TAG=$1; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SEL=${*:-tests}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -2 "$OUT/pytest_gpu.log"
grep -E "^FAILED|^ERROR" "$OUT/pytest_gpu.log" | head -30
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc;; esac
if [ -n "${AB:-}" ]; then
  for rep in 1 2; do for v in intree $AB; do
    if [ $v = intree ]; then LP=""; else LP=$GRAFT_REPO_ROOT/tools/_abl/liblgnn_$v.so; fi
    LGNN_LIB_PATH=$LP timeout -k 10 200 python bench.py --workload ${W:-c2} --steps 300 --warmup 30 \
      --cpu-seconds 0 > "$OUT/ab_${v}_$rep.json" 2> "$OUT/ab_${v}_$rep.err" || { tail -20 "$OUT/ab_${v}_$rep.err"; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d.get('roofline',{}).get('avg_launch_ms'), [r.get('avg_launch_ms') for r in d.get('roofline_next',[])])"
  done; done
fi
exit $rc
