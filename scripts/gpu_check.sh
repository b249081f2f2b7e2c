set -o pipefail
mkdir -p gpurun_out/r9
timeout -k 10 600 python -m pytest tests -m gpu -x -v > gpurun_out/r9/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r9/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r9/pytest_gpu.log
for a in "" "--graph" "--loopback --periodic" "--loopback --periodic --graph"; do
  timeout -k 10 180 python bench.py --steps 200 --warmup 20 $a > gpurun_out/r9/bench_$(echo $a | tr -d ' -').log 2>&1 || { echo BENCH_FAIL $a; tail -20 gpurun_out/r9/bench_$(echo $a | tr -d ' -').log; exit 1; }
  echo "== $a"; tail -1 gpurun_out/r9/bench_$(echo $a | tr -d ' -').log
done
