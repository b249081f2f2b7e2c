set -o pipefail
mkdir -p gpurun_out/r11
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r11/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r11/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r11/pytest_gpu.log
IGG_TRANSPORT=put timeout -k 10 100 python benchmarks/halo_only.py --reps 50 2>&1 | grep halo_us
for t in rccl put; do for g in "" "--graph"; do
  IGG_TRANSPORT=$t timeout -k 10 180 python bench.py --steps 200 --warmup 20 --loopback --periodic $g > gpurun_out/r11/bench_lb_$t$g.log 2>&1 || { echo BENCH_FAIL $t $g; tail -20 gpurun_out/r11/bench_lb_$t$g.log; exit 1; }
  echo "== $t $g $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r11/bench_lb_$t$g.log)"
done; done
