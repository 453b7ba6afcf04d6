#!/bin/bash
# A/B baseline for the stamps / in-step tools: the library built from a git revision's sources
# (default HEAD) as tools/_abl/liblgnn_s3f_base.so and liblgnn_s3f_base_stamps.so.
# Usage (here, not on the GPU box): bash tools/build_base_lib.sh [rev]
set -euo pipefail
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" lesion_gnn_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$ROOT/tools/_abl"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared -I$TMP/include"
/opt/rocm/bin/hipcc $F "$TMP"/lesion_gnn_amd/csrc/*.hip -o "$ROOT/tools/_abl/liblgnn_s3f_base.so" &
/opt/rocm/bin/hipcc $F -DLGNN_STAMPS "$TMP"/lesion_gnn_amd/csrc/*.hip -o "$ROOT/tools/_abl/liblgnn_s3f_base_stamps.so" &
wait
rm -rf "$TMP"
