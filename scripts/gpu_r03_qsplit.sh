#!/bin/bash
# Verify-attention query split (attention_kernel QS == 2): GPU tests, then the
# per-rank TP shard bench at TP 8 / 4 / 2 with FFMI_ATTN_QSPLIT=0 / 1 (same box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
run() { local n=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || tail -n 30 "gpurun_out/$n.log"; return $rc; }
run t_qs 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py tests/test_gpu_tp_local.py -x -q --timeout 200 --timeout-method thread && \
run qs0_tp8 300 env FFMI_ATTN_QSPLIT=0 python scripts/tp_shard_bench.py --tp 8 && tail -1 gpurun_out/qs0_tp8.log && \
run qs1_tp8 300 env FFMI_ATTN_QSPLIT=1 python scripts/tp_shard_bench.py --tp 8 && tail -1 gpurun_out/qs1_tp8.log && \
run qs0_tp4 300 env FFMI_ATTN_QSPLIT=0 python scripts/tp_shard_bench.py --tp 4 && tail -1 gpurun_out/qs0_tp4.log && \
run qs1_tp4 300 env FFMI_ATTN_QSPLIT=1 python scripts/tp_shard_bench.py --tp 4 && tail -1 gpurun_out/qs1_tp4.log && \
run qs0_tp2 300 env FFMI_ATTN_QSPLIT=0 python scripts/tp_shard_bench.py --tp 2 && tail -1 gpurun_out/qs0_tp2.log && \
run qs1_tp2 300 env FFMI_ATTN_QSPLIT=1 python scripts/tp_shard_bench.py --tp 2 && tail -1 gpurun_out/qs1_tp2.log && \
run qs1b_tp8 300 env FFMI_ATTN_QSPLIT=1 python scripts/tp_shard_bench.py --tp 8 && tail -1 gpurun_out/qs1b_tp8.log && \
run qs0b_tp8 300 env FFMI_ATTN_QSPLIT=0 python scripts/tp_shard_bench.py --tp 8 && tail -1 gpurun_out/qs0b_tp8.log
