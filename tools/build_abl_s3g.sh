#!/bin/bash
# timing-ablation builds of s3gemm.hip (tools/_abl/liblgnn_v_<bits>.so): bit 1 = no MFMA,
# 2 = no global loads in the chunk loop. Here, not on the GPU box.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/tools/_abl" "$ROOT/build_ab"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950"
for b in "$@"; do
  /opt/rocm/bin/hipcc $F -DLGNN_ABL_S3G=$b -c "$ROOT/lesion_gnn_amd/csrc/s3gemm.hip" -o "$ROOT/build_ab/s3gemm_$b.o"
  objs=$(ls "$ROOT"/build/*.o | grep -v '/s3gemm.o$')
  /opt/rocm/bin/hipcc $F -shared $objs "$ROOT/build_ab/s3gemm_$b.o" -o "$ROOT/tools/_abl/liblgnn_v_$b.so"
done
