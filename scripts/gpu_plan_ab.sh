# A/B of forced M-split GEMM plans (FFMI_GEMM_PLAN="NTW,S") at T=168, cold weights.
set -o pipefail
mkdir -p gpurun_out
run() {
  echo "== plan ${1:-default} ops $2" >> gpurun_out/plan_ab.log
  FFMI_GEMM_PLAN=$1 timeout -k 10 120 python scripts/gemm_bench.py --T 168 --xpacked --ops $2 >> gpurun_out/plan_ab.log 2>&1
}
: > gpurun_out/plan_ab.log
run "" qkv,o,gate_up,down,lm_head && \
run 6,2 gate_up && run 8,2 gate_up && run 12,2 gate_up && run 16,2 gate_up && run 16,4 gate_up && \
run 6,1 qkv && run 12,2 qkv && run 12,4 qkv && run 16,4 qkv && \
run 8,4 o && run 16,4 o && run 6,8 o && run 16,8 o && \
run 8,4 down && run 16,4 down && run 16,8 down && run 6,8 down
rc=$?
cat gpurun_out/plan_ab.log | grep -v Warn
exit $rc
