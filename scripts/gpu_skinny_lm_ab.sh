set -o pipefail
mkdir -p gpurun_out
for v in "" "4,4" "4,2" "2,8" "2,2" "1,8"; do
  echo "== FFMI_SKINNY=$v" >> gpurun_out/ssm_lm_ab.log
  FFMI_SKINNY=$v timeout -k 10 120 python -u scripts/gemm_bench.py --shapes ssm --T 8,24 --ops lm_head,qkv,gate_up --cold-mb 0 >> gpurun_out/ssm_lm_ab.log 2>&1 || exit 1
done
