#!/bin/bash
# Round 6: the SSM lm_head's wave GEMM forms (FFMI_WAVE_FORM=NT,WPG: tiles per
# wave, waves per workgroup) standalone at T = 8 / 24 and in the bench's SSM
# step, same box, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
OUT=gpurun_out/r06_wave_gemm.log
: > $OUT
for rep in 1 2; do
  for f in 2,4 4,2 4,4 3,2 2,2; do
    echo "form $f" >> $OUT
    FFMI_WAVE_FORM=$f timeout -k 10 120 python scripts/gemm_bench.py --shapes ssm --ops lm_head --T 8,24 >> $OUT 2>gpurun_out/wave.err || { tail -5 gpurun_out/wave.err; exit 1; }
  done
done
cat $OUT
bash scripts/gpu_ab.sh -r 2 "" "FFMI_WAVE_FORM=4,2" "FFMI_WAVE_FORM=4,4"
