set -uo pipefail
mkdir -p gpurun_out/r03h15
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --cpu-seconds 0 > gpurun_out/r03h15/bench.json 2> gpurun_out/r03h15/bench.err || { tail -20 gpurun_out/r03h15/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r03h15/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['kernel'][:30], r['avg_launch_ms'], r['frac'])"
PATTERN=k_s3_fbwd bash tools/ab_prof.sh xearly --workload c2
