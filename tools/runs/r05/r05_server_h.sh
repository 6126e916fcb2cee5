#!/bin/bash
# Round 5: staging of pageable bursts at many threads: device memory over the
# BAR (CPU stores) vs pinned host memory the GPU reads over PCIe; one server
# block per CU (96 KiB of dynamic LDS).
set -o pipefail
O=gpurun_out/${R05_OUT:-r05h}
mkdir -p $O
run() {   # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 240 python -u tools/server_scaling.py > $O/ss_$name.json 2> $O/ss_$name.err
}
C="SS_THREADS=1,4,8,12,16 SS_RINGS=4x4,4x6 SS_ITERS=400 GCS_SERVER_LDS_KB=96"
for rep in 1 2; do
    run dev_r$rep SS_PROF=0 GCS_DIRECT_STAGE=device $C || exit 1
    run host_r$rep SS_PROF=0 GCS_DIRECT_STAGE=host GCS_ASYNC_STAGE=host $C || exit 1
done
run host_prof GCS_DIRECT_STAGE=host GCS_ASYNC_STAGE=host $C || exit 1
