set -uo pipefail
mkdir -p gpurun_out/r03h23
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_gcn.py tests/test_gpu_configs.py tests/test_gpu_gat.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03h23/pt.log 2>&1
rc=$?; tail -2 gpurun_out/r03h23/pt.log; grep -E "^FAILED|^ERROR" gpurun_out/r03h23/pt.log | head -20
case $rc in 0) ;; *) exit $rc;; esac
PATTERN=k_ bash tools/ab_prof.sh base --workload c2 2>&1 | python3 -c "
import sys,ast
for line in sys.stdin:
    v,rest=line.split(' ',1)
    lst,ms=rest.rsplit(' ',1)
    d=dict(ast.literal_eval(lst))
    print(v, ms.strip(), {k[:30]:x for k,x in d.items() if any(t in k for t in ('prep','count','scan','fill','finish'))})
"
