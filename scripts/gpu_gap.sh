# Autotune vs timed-loop gap of the 1-GPU stencil (benchmarks/loop_gap.py).
set -o pipefail
O=gpurun_out/gap; mkdir -p $O
timeout -k 10 300 python benchmarks/loop_gap.py > $O/auto.log 2>&1 || { echo FAIL; tail -20 $O/auto.log; exit 1; }
tail -1 $O/auto.log
timeout -k 10 200 python benchmarks/loop_gap.py --variant 40 > $O/v40.log 2>&1 || { echo FAIL; tail -20 $O/v40.log; exit 1; }
tail -1 $O/v40.log
