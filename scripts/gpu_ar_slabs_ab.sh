# one-GPU N-rank rehearsal A/B: slabs into the all-reduce copy-in vs reduce pass
set -o pipefail
mkdir -p gpurun_out
(while true; do date >> gpurun_out/rehearsal_heartbeat.log; sleep 30; done) &
HB=$!
rc=0
for v in ${VALS:-1 0}; do
  env ${VAR:-FFMI_AR_SLABS}=$v FFMI_BENCH_DEVICE=0 FFMI_TP_TRANSPORT=xgmi-only timeout -k 10 300 python bench.py --gpus ${N:-4} --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/arslab_$v.log 2>&1 || { echo "${VAR:-FFMI_AR_SLABS}=$v failed"; tail -20 gpurun_out/arslab_$v.log; rc=1; break; }
  grep '^{' gpurun_out/arslab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('${VAR:-FFMI_AR_SLABS}=$v', d['value'], d['verify_step_ms'], d['ssm_step_us'], {k: v['avg_us'] for k, v in d['op_breakdown_sampled'].items()})"
done
kill $HB
exit $rc
