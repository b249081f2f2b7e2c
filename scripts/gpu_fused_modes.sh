# A/B of the fused kernel designs (IGG_FUSED_MODE 0..3) per variant.
set -o pipefail
export IGG_PUT_TIMEOUT=10
O=gpurun_out/fused; mkdir -p $O
for m in 0 1 2 3; do
  IGG_FUSED_MODE=$m timeout -k 10 240 python benchmarks/fused_sweep.py --variants ${VARIANTS:-0,2,9,11,14} > $O/modes_$m.log 2>&1 || { echo SWEEP_FAIL $m; tail -20 $O/modes_$m.log; exit 1; }
  echo "== mode $m"; grep variant $O/modes_$m.log
done
