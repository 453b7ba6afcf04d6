set -uo pipefail
export TMPDIR=/tmp
bash tools/gpu_cmd2.sh || exit 1
bash tools/gpu_suite.sh r03h30 || exit 1
WL="c2 refcfg" BW="c2 refcfg c3 c3f32 c4 c5k4 c5k16" bash tools/gpu_r03_final.sh r03h30f
