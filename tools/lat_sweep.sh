#!/bin/bash
# Burst-server latency under its knobs (GPU box; tools/, not product).
set -o pipefail
for P in 1 2; do
  GCS_SERVER_POLLERS=$P timeout -k 10 120 python tools/lat_probe.py > gpurun_out/lat_p$P.json 2>gpurun_out/lat_p$P.err || exit 1
  GCS_SERVER_PROF=1 GCS_SERVER_POLLERS=$P timeout -k 10 120 python tools/lat_probe.py > /dev/null 2>gpurun_out/lat_p${P}_prof.err || exit 1
done
