#!/bin/bash
# Round 5: rocprofv3 evidence after the wide LRO -- the C2ext configurations
# (copy + fill, LRO 64 and 256) traced and counted in separate passes, and
# bench.py with its side measurements under --stats.
set -o pipefail
OUT=gpurun_out/prof_r05w
mkdir -p "$OUT"
CFG="python3 profiles/pmc_configs.py --reps 5 --configs C2ext"
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
