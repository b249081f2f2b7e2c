# Fused selection with a bitwise check of the kept candidate: loopback xyz/xy, 2-rank share-gpu.
set -o pipefail
O=gpurun_out/fsel; mkdir -p $O
for p in xyz xy; do
timeout -k 10 400 python bench.py --loopback --periodic-dims $p --steps 50 --warmup 5 > $O/lb_$p.log 2>&1 || { echo LB_FAIL; tail -30 $O/lb_$p.log; exit 1; }
grep -E "fused A/B|fused check" $O/lb_$p.log | cut -c1-900; tail -1 $O/lb_$p.log | cut -c1-150
done
timeout -k 10 300 python bench.py --gpus 2 --share-gpu --n 192 --steps 50 --warmup 5 --launch-timeout 250 > $O/b2.log 2>&1 || { echo B2_FAIL; tail -30 $O/b2.log; exit 1; }
grep -E "fused A/B|validation" $O/b2.log | cut -c1-500; tail -1 $O/b2.log | cut -c1-150
