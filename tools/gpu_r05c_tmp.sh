set -uo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > $O/list.txt 2>&1; grep -i -B2 -A12 "pc.sampl\|PC_SAMPL" $O/list.txt | head -60
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 65536 --kernel-include-regex k_s3_fbwd -d $O/pcs -o pcs --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/fbwd_loop.py 100 > $O/pcs.log 2>&1; echo "rc=$?"; tail -5 $O/pcs.log; find $O/pcs -type f | head; 
