#!/bin/bash
# Round-5 bottleneck counters of the verify-step gate/up GEMM (T = 168,
# gemm_mid_kernel<3,6,4,1,...>) and of the xl2 probe's loop (modes 7 and 1):
# TA / TD busy and stall cycles, TCP stalls and requests, SQ instruction mix and
# wait states.  One rocprofv3 --pmc pass per counter group (slot limits:
# SQ 8, TA 2, TD 2, TCP 4, GRBM 2), each under its own kill timeout.
#   scripts/r05_pmc_gemm.sh   -> gpurun_out/r05_pmc/*.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/r05_pmc
export TMPDIR=/tmp
O=gpurun_out/r05_pmc
hipcc --offload-arch=gfx950 -O3 -o /tmp/xl2_probe scripts/probe/xl2_probe.hip || exit 1
PASSES=(
  "TA_BUSY_avr TA_BUSY_max TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
  "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum GRBM_GUI_ACTIVE"
  "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
  "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_F16"
  "SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
)
GEMM="python3 $R/scripts/gemm_bench.py --shapes llama7b --ops gate_up --T 168 --xpacked --wstream --iters 30"
n=0
for P in "${PASSES[@]}"; do
  echo "== pass $n: $P"
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/pmc_g$n -o g -- $GEMM \
     > "$R/$O/gemm_$n.log" 2>&1) || { echo "gemm pass $n failed"; tail -5 "$O/gemm_$n.log"; exit 1; }
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d /tmp/pmc_p$n -o p -- /tmp/xl2_probe rnd \
     > "$R/$O/probe_$n.log" 2>&1) || { echo "probe pass $n failed"; tail -5 "$O/probe_$n.log"; exit 1; }
  n=$((n + 1))
done
python3 scripts/pmc_counters.py $O/gemm_counters.json "ffmi::gemm_mid_kernel" /tmp/pmc_g* > /dev/null
python3 scripts/pmc_counters.py $O/probe_counters.json "probe" /tmp/pmc_p* > /dev/null
tail -3 $O/gemm_0.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt -o k -- $GEMM > $O/gemm_kt.log 2>&1 \
  && cp /tmp/kt/k_kernel_stats.csv $O/gemm_kernel_stats.csv
echo done
