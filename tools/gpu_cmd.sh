set -uo pipefail
mkdir -p gpurun_out/r03h7
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_gcn.py tests/test_gpu_gat.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03h7/pt.log 2>&1
rc=$?; tail -2 gpurun_out/r03h7/pt.log; grep -E "^FAILED|^ERROR" gpurun_out/r03h7/pt.log | head -20
case $rc in 0) ;; *) exit $rc;; esac
bash tools/ab_lib.sh base --workload c2
bash tools/ab_lib.sh base --workload refcfg
