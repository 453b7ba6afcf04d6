#!/bin/bash
# r03k: SQ counter passes on refcfg + wgrad split sweep
set -uo pipefail
OUT=gpurun_out/r03k; mkdir -p $OUT
bash tools/pmc_sq.sh r03k refcfg > $OUT/sqA.txt 2>&1 || exit 1
COUNTERS="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" SUB=sqB bash tools/pmc_sq.sh r03k refcfg > $OUT/sqB.txt 2>&1 || exit 1
for mc in 4 8 12 16; do
  LGNN_S3_WG_MINCPS=$mc timeout -k 10 200 python bench.py --workload refcfg --steps 200 --warmup 30 --cpu-seconds 0 > $OUT/mc$mc.json 2>$OUT/mc$mc.err || exit 1
  python -c "import json; d=json.load(open('$OUT/mc$mc.json')); print('mincps', $mc, d['ms_per_step'])"
done
