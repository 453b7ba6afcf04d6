set -e
mkdir -p gpurun_out/ab
for v in "1 0" "0 0" "1 0" "0 0"; do set -- $v
LGNN_HEAD_FOLD=$1 LGNN_HEAD_SIDE=$2 timeout -k 10 200 python bench.py --steps 300 --warmup 30 --cpu-seconds 0 > gpurun_out/ab/b_$1$2.json
python -c "import json,sys; d=json.loads(open('gpurun_out/ab/b_$1$2.json').read().strip().splitlines()[-1]); print('fold=$1 side=$2', d['ms_per_step'])"
done
