set -uo pipefail
mkdir -p gpurun_out/r03h29
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_gcn.py tests/test_gpu_gat.py tests/test_gpu_gin.py tests/test_gpu_configs.py tests/test_gpu_drgnet.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03h29/pt.log 2>&1
rc=$?; tail -2 gpurun_out/r03h29/pt.log; grep -E "^FAILED|^ERROR" gpurun_out/r03h29/pt.log | head -20
case $rc in 0) ;; *) exit $rc;; esac
for w in refcfg c5k16 c5k4; do
PATTERN=k_ bash tools/ab_prof.sh base --workload $w 2>&1 | python3 -c "
import sys,ast
for line in sys.stdin:
    v,rest=line.split(' ',1)
    lst,ms=rest.rsplit(' ',1)
    d=dict(ast.literal_eval(lst))
    print('$w', v, ms.strip(), {k[22:34]:x for k,x in d.items() if any(t in k for t in ('k_count','k_fill','k_finish','k_scan','k_prep'))})
"
done
