#!/bin/bash
# profiles/collect.sh ROUND -- rocprofv3 evidence for bench.py's kernels (run on the GPU box).
#
#   1. --kernel-trace --stats           : per-kernel durations (must agree with bench.py's HIP events)
#   2. --pmc FETCH_SIZE  (own pass)     : HBM read KB per dispatch
#   3. --pmc WRITE_SIZE  (own pass)     : HBM write KB per dispatch
# Counters are collected in their own runs with --kernel-trace only (no sys/hip
# traces beside --pmc).  profiles/summarize.py then applies the gfx950
# correction (FETCH_SIZE reports 1/2 of a wide streaming read:
# MI355X_MICROARCH.md §HBM) and writes profiles/pmc_summary.json.
set -o pipefail
ROUND=${1:-r01}
OUT=gpurun_out/prof_$ROUND
mkdir -p "$OUT"
CMD="python bench.py --steps 10 --warmup 2 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- $CMD > "$OUT/trace.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run \
    -- $CMD > "$OUT/fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run \
    -- $CMD > "$OUT/write.log" 2>&1
# then, back in the build container (gpurun merges gpurun_out/):
#   python profiles/summarize.py gpurun_out/prof_$ROUND $ROUND
