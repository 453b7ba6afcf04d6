set -uo pipefail
O=gpurun_out/r05i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_weight_planes.py tests/test_gpu_graph_build.py tests/test_gpu_pool.py tests/test_gpu_ce_fused.py tests/test_gpu_gcn.py tests/test_gpu_s3.py tests/test_gpu_gin.py tests/test_gpu_optim.py tests/test_gpu_compile.py tests/test_gpu_radius.py tests/test_gpu_configs.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 1; }
for w in c2 c5k16; do
timeout -k 10 300 python bench.py --workload $w --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $O/$w.json 2> $O/$w.err || { tail $O/$w.err; exit 1; }
python -c "import json; d=json.loads(open('$O/$w.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$w', d['value'], d['ms_per_step'], r.get('avg_launch_ms'), r.get('frac'), [(e['entry'], e['avg_launch_ms']) for e in d.get('entries', [])][:14])"
done
