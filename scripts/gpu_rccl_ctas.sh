# RCCL workgroup cap (IGG_RCCL_MAX_CTAS) vs the overlapped step, interior rank emulated (loopback, RCCL transport).
set -o pipefail
O=gpurun_out/ctas; mkdir -p $O
for c in "" 1 2 4 16; do
  IGG_TRANSPORT=rccl IGG_RCCL_MAX_CTAS=$c timeout -k 10 200 python bench.py --loopback --periodic --overlap --fused off --no-graph --steps 100 --warmup 10 > $O/ov_$c.log 2>&1 || { echo FAIL $c; tail -20 $O/ov_$c.log; exit 1; }
  grep '^{' $O/ov_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('overlap max_ctas=${c:-default}', d['ms_per_step'], d['config'].get('phase_ms'))"
done
for c in "" 2; do
  IGG_TRANSPORT=rccl IGG_RCCL_MAX_CTAS=$c timeout -k 10 200 python bench.py --loopback --periodic --fused off --transport rccl --steps 100 --warmup 10 > $O/seq_$c.log 2>&1 || { echo FAIL seq $c; tail -20 $O/seq_$c.log; exit 1; }
  grep '^{' $O/seq_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('no-overlap max_ctas=${c:-default}', d['ms_per_step'], d['config'].get('phase_ms'))"
done
