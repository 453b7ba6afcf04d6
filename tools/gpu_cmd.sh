set -uo pipefail
mkdir -p gpurun_out/r03h3
export TMPDIR=/tmp
timeout -k 10 300 python tools/stamps_s3f.py run > gpurun_out/r03h3/stamps.txt 2>&1 || { tail -20 gpurun_out/r03h3/stamps.txt; exit 1; }
cat gpurun_out/r03h3/stamps.txt
bash tools/ab_lib.sh base --workload c2
