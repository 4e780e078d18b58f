#!/bin/bash
# Round 6: decode fused-norm consumer GEMMs with 8 K-split waves
# (FFMI_FZ_KW8=1: qkv; 2: qkv and gate/up) vs 4, incremental decoding,
# same box, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
bash scripts/gpu_ab.sh -r 3 -b "--mode incr --no-legs" "" "FFMI_FZ_KW8=1" "FFMI_FZ_KW8=2"
