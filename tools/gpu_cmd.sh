set -uo pipefail
mkdir -p gpurun_out/r03h26
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_gcn.py tests/test_gpu_configs.py tests/test_gpu_gat.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03h26/pt.log 2>&1
rc=$?; tail -2 gpurun_out/r03h26/pt.log; grep -E "^FAILED|^ERROR" gpurun_out/r03h26/pt.log | head -20
case $rc in 0) ;; *) exit $rc;; esac
PATTERN=k_pool bash tools/ab_prof.sh base --workload c2
PATTERN=k_pool bash tools/ab_prof.sh base --workload refcfg
