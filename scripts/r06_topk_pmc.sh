#!/bin/bash
# Round 6: counters of the softmax top-k (scripts/topk_bench.py shapes): wave
# time split into VALU issue and waits, and the fetched bytes, one rocprofv3
# --pmc pass per counter group.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
P=/tmp/ffmi_topk_pmc
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $P/sq -o tk -- python3 scripts/topk_bench.py > gpurun_out/topk_pmc_sq.log 2>&1 || { tail -5 gpurun_out/topk_pmc_sq.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o tk -- python3 scripts/topk_bench.py > gpurun_out/topk_pmc_fetch.log 2>&1 || { tail -5 gpurun_out/topk_pmc_fetch.log; exit 1; }
python3 scripts/pmc_counters.py gpurun_out/r06_topk_pmc.json ffmi::softmax_topk_reg_kernel $P/sq $P/fetch && head -c 3000 gpurun_out/r06_topk_pmc.json
