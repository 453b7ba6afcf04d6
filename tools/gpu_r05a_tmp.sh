set -uo pipefail
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/stamps_s3f.py run > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
cat $O/stamps.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 > $O/c2_drv.json 2> $O/c2_drv.err || { tail $O/c2_drv.err; exit 1; }
python -c "import json; d=json.loads(open('$O/c2_drv.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(d['value'], d['ms_per_step'], r.get('avg_launch_ms'), r.get('frac'), [(e['entry'], e['avg_launch_ms']) for e in d.get('entries', [])][:14])"
