#!/bin/bash
# profiles/collect.sh ROUND -- rocprofv3 evidence for bench.py's kernels (run on the GPU box).
#
#   bench/  --kernel-trace --stats of bench.py itself (the bench line's command):
#           its per-kernel averages must agree with the line's HIP-event times
#   trace/  --kernel-trace of profiles/pmc_configs.py (per-configuration launches)
#   fetch/  --pmc FETCH_SIZE of the same command (own pass)
#   write/  --pmc WRITE_SIZE of the same command (own pass)
#   bench_extras/  --kernel-trace --stats of bench.py WITH its side measurements
#           (C1, C3, rows_8f ...): the side kernels' averages from the command
#           whose JSON line reports them
# Counters are collected in their own runs with --kernel-trace only (no sys/hip
# traces beside --pmc).  Back in the build container (gpurun merges gpurun_out/):
#   python profiles/summarize.py gpurun_out/prof_$ROUND $ROUND
set -o pipefail
ROUND=${1:-r02}
OUT=gpurun_out/prof_$ROUND
mkdir -p "$OUT"
CFG="python3 profiles/pmc_configs.py --reps 5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o run \
    -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extras > "$OUT/bench.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run \
    -- $CFG --manifest "$OUT/manifest.json" > "$OUT/trace.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run \
    -- $CFG > "$OUT/fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run \
    -- $CFG > "$OUT/write.log" 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench_extras" -o run \
    -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 > "$OUT/bench_extras.log" 2>&1
