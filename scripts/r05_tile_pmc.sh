#!/bin/bash
# Tile GEMM (prefill, T = 1024) A/B against the M-split kernel, then its SQ
# wait / LDS / MFMA counters (one --pmc pass) -> gpurun_out/r05_tile_pmc.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="scripts/gemm_bench.py --shapes llama7b --ops qkv,gate_up,lm_head --T 1024 --xpacked --wstream --iters 20"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_llama_shapes.py -k tile_gemm > gpurun_out/tile_test.log 2>&1 || { tail -30 gpurun_out/tile_test.log; exit 1; }
tail -2 gpurun_out/tile_test.log
# (round 5 also ran a register-staged arm, FFMI_TILE_GEMM=3, since removed:
# profiles/r05_tile_gemm_variants_ab.log)
bash scripts/gpu_kernel_ab.sh "$CMD" "" "FFMI_TILE_GEMM=0" "" || exit 1
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
   --output-format csv -d /tmp/tpmc -o t -- python3 $R/$CMD > $R/gpurun_out/tile_pmc.log 2>&1) || { tail -5 gpurun_out/tile_pmc.log; exit 1; }
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TD_TD_BUSY_sum TD_TC_STALL_sum \
   --output-format csv -d /tmp/tpmc2 -o t -- python3 $R/$CMD > $R/gpurun_out/tile_pmc2.log 2>&1) || { tail -5 gpurun_out/tile_pmc2.log; exit 1; }
python3 scripts/pmc_counters.py gpurun_out/r05_tile_pmc.json "ffmi::gemm_tile_kernel" /tmp/tpmc /tmp/tpmc2 > /dev/null
python3 -c "
import json; d=json.load(open('gpurun_out/r05_tile_pmc.json'))
for r in d: print(r['kernel'], r['grid_size'], {k:v for k,v in r.items() if 'frac' in k or 'of_wave' in k})"
