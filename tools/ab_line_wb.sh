set -e
mkdir -p gpurun_out/ab_wb
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 50 --no-extras > gpurun_out/ab_wb/line_$r.json 2>/dev/null
  GCS_TX_LINE_WB_MB=0 timeout -k 10 120 python bench.py --steps 50 --no-extras > gpurun_out/ab_wb/sector_$r.json 2>/dev/null
done
