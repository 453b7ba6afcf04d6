set -uo pipefail
mkdir -p gpurun_out/r03h12
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gcn.py tests/test_lib.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r03h12/pt.log 2>&1
rc=$?; tail -2 gpurun_out/r03h12/pt.log; grep -E "^FAILED|^ERROR|s3f8" gpurun_out/r03h12/pt.log | head -20
case $rc in 0) ;; *) exit $rc;; esac
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03h12/prof_c5k16 -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5k16 --steps 20 --warmup 5 --cpu-seconds 0 --no-kernel-timing > $GRAFT_REPO_ROOT/gpurun_out/r03h12/c5k16.json 2> $GRAFT_REPO_ROOT/gpurun_out/r03h12/c5k16.err || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r03h12/c5k16.err; exit 1; }
echo c5 prof done
