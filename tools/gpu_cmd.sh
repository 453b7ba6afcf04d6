set -uo pipefail
mkdir -p gpurun_out/r03h8
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_s3gemm.py tests/test_gpu_gat.py tests/test_gpu_gat_pipe.py tests/test_gpu_configs.py tests/test_gpu_compile.py tests/test_gpu_dropout.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r03h8/pt.log 2>&1
rc=$?; tail -2 gpurun_out/r03h8/pt.log; grep -E "^FAILED|^ERROR" gpurun_out/r03h8/pt.log | head -20
case $rc in 0) ;; *) exit $rc;; esac
VAR=LGNN_S3G_HALF A=0 B=1 W="refcfg c3f32" STEPS=150 bash tools/gpu_ab.sh r03h8
