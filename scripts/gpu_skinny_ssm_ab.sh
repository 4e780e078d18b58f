set -o pipefail
for v in "" "4,4" "4,2" "2,8" "2,2" "1,8"; do
  echo "== FFMI_SKINNY='$v'"
  FFMI_SKINNY=$v timeout -k 10 100 python scripts/gemm_bench.py --shapes ssm --T 24 --cold-mb 0 --iters 50 || exit 1
done
