# N-rank bench rehearsal on ONE GPU (ranks time-share the device over the
# xGMI-transport code path; checks the multi-rank path, not its speed).
# GPU_MAX_HW_QUEUES=1: N ranks x HIP's default 4 hardware queues oversubscribe
# the device and the scheduler time-slices processes (TP 8: 370 s per
# generate, 7.6 s with one queue per rank); never set on a real N-GPU node.
# A heartbeat file marks the run alive (N ranks on one device take minutes);
# every rehearsal is still bounded by its own timeout.
set -o pipefail
mkdir -p gpurun_out
(while true; do date >> gpurun_out/rehearsal_heartbeat.log; sleep 30; done) &
HB=$!
rc=0
for n in ${NS:-2 8}; do
  GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-1} FFMI_BENCH_DEVICE=0 FFMI_TP_TRANSPORT=xgmi-only timeout -k 10 ${TMO:-600} python bench.py --gpus $n --steps 1 --warmup ${WARM:-0} --no-cpu-baseline > gpurun_out/rehearsal_tp$n.log 2>&1 || { echo "tp$n failed"; tail -20 gpurun_out/rehearsal_tp$n.log; rc=1; break; }
  grep '^{' gpurun_out/rehearsal_tp$n.log | tail -1 > gpurun_out/${TAG:-r03}_rehearsal_tp${n}_one_gpu.json
  cut -c1-300 gpurun_out/${TAG:-r03}_rehearsal_tp${n}_one_gpu.json
done
kill $HB
exit $rc
