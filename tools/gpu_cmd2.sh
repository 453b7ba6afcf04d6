set -uo pipefail
mkdir -p gpurun_out/r03h31
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph_build.py tests/test_gpu_gcn.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03h31/pt.log 2>&1
rc=$?; tail -2 gpurun_out/r03h31/pt.log; grep -E "^FAILED|^ERROR" gpurun_out/r03h31/pt.log | head -20
case $rc in 0) ;; *) exit $rc;; esac
for w in c5k16 c5k4; do
PATTERN=k_finish bash tools/ab_prof.sh base --workload $w
done
