#!/bin/bash
# One GPU session of round profiles: bench line, rocprofv3 kernel stats (csv),
# PMC fetch, PMC MFMA utilisation (each counter pass in its own run), the
# per-rank TP shard table and the incr-decoding kernel stats.  Raw rocprofv3
# output stays in /tmp on the box; the summaries land in gpurun_out/ (gpurun
# copies back at most 64 MiB), to be copied into profiles/.
#
# rocprofv3 runs with DEBUG_CLR_GRAPH_PACKET_CAPTURE=0: with HIP's default
# graph packet capture, the tracer segfaults inside hipGraphLaunch (the
# tracer's AQL-packet intercept reads past the end of a 1 MiB queue mapping
# when a replay submits its batch of packets).  With it off the
# graphed steps are traced like the bench runs them (same kernels, same
# graphs; the packets go out one by one).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-r02}
P=/tmp/ffmi_prof_$TAG
B="$R/bench.py --steps 1 --no-cpu-baseline --no-incr --no-legs --profile 0"
run() { local n=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || tail -n 20 "gpurun_out/$n.log"; return $rc; }
run bench 400 python bench.py && grep '^{' gpurun_out/bench.log | tail -1 > "gpurun_out/${TAG}_bench.json" && \
(export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0; cd /tmp && \
 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/prof" -o bench -- python3 $B --warmup 1 > "$R/gpurun_out/prof.log" 2>&1 && \
 cp "$P/prof/bench_kernel_stats.csv" "$R/gpurun_out/${TAG}_bench_kernel_stats.csv" && echo "[prof] ok" && \
 timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/pmc" -o bench -- python3 $B --warmup 0 > "$R/gpurun_out/pmc.log" 2>&1 && \
 python3 "$R/scripts/pmc_summary.py" "$P/pmc/bench_counter_collection.csv" > "$R/gpurun_out/${TAG}_pmc_fetch.json" && \
 python3 "$R/scripts/pmc_table.py" "$P/pmc/bench_counter_collection.csv" > "$R/gpurun_out/${TAG}_pmc_fetch_table.json" && echo "[pmc] ok" && \
 timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$P/pmcw" -o bench -- python3 $B --warmup 0 > "$R/gpurun_out/pmc_w.log" 2>&1 && \
 python3 "$R/scripts/pmc_table.py" "$P/pmcw/bench_counter_collection.csv" > "$R/gpurun_out/${TAG}_pmc_write_table.json" && echo "[pmc write] ok" && \
 timeout -k 10 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$P/mfma" -o bench -- python3 $B --warmup 0 > "$R/gpurun_out/pmc_mfma.log" 2>&1 && \
 python3 "$R/scripts/mfma_summary.py" "$P/mfma/bench_counter_collection.csv" > "$R/gpurun_out/${TAG}_pmc_mfma.json" && echo "[pmc_mfma] ok" && \
 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/incr" -o incr -- python3 "$R/bench.py" --mode incr --steps 1 --warmup 1 --no-cpu-baseline --no-legs --profile 0 > "$R/gpurun_out/incr_prof.log" 2>&1 && \
 cp "$P/incr/incr_kernel_stats.csv" "$R/gpurun_out/${TAG}_incr_kernel_stats.csv" && echo "[incr prof] ok") && \
{ [ "${SKIP_AUX:-0}" = 1 ] || TAG=$TAG bash scripts/gpu_refresh_aux.sh; }
