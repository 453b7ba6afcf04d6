set -uo pipefail
mkdir -p gpurun_out/r03h27
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_gat.py tests/test_gpu_gat_pipe.py tests/test_gpu_compile.py tests/test_gpu_dropout.py tests/test_gpu_configs.py tests/test_gpu_s3gemm.py tests/test_gpu_golden.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03h27/pt.log 2>&1
rc=$?; tail -2 gpurun_out/r03h27/pt.log; grep -E "^FAILED|^ERROR" gpurun_out/r03h27/pt.log | head -20
case $rc in 0) ;; *) exit $rc;; esac
for rep in 1 2; do
  for v in new base; do
    if [ $v = base ]; then cp tools/_abl/ops_base.py lesion_gnn_amd/ops.py; else cp tools/_abl/ops_new.py lesion_gnn_amd/ops.py; fi
    timeout -k 10 300 python bench.py --workload refcfg --steps 150 --warmup 30 --cpu-seconds 0 --no-kernel-timing > gpurun_out/r03h27/$v$rep.json 2> gpurun_out/r03h27/$v$rep.err || { tail -5 gpurun_out/r03h27/$v$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r03h27/$v$rep.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'])"
  done
done
cp tools/_abl/ops_new.py lesion_gnn_amd/ops.py
