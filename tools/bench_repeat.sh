# bench.py at its defaults, three times on one box (run-to-run spread of the bench line)
set -e
mkdir -p gpurun_out/bench_repeat
for r in 1 2 3; do
  timeout -k 10 240 python bench.py > gpurun_out/bench_repeat/bench_$r.json 2> gpurun_out/bench_repeat/bench_$r.err
done
