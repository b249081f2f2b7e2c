# Arena memory kind A/B for the fused exchange (loopback periodic interior rank) + per-face pack cost.
set -o pipefail
O=gpurun_out/arena; mkdir -p $O
timeout -k 10 120 python benchmarks/pack_faces.py > $O/pack_faces.log 2>&1 || { echo PACK_FAIL; tail -20 $O/pack_faces.log; exit 1; }
cat $O/pack_faces.log | grep -v amdgpu.ids
for k in 3 1 0; do
IGG_PUT_ARENA_KIND=$k timeout -k 10 300 python bench.py --loopback --periodic --steps 100 --warmup 10 > $O/lb_kind$k.log 2>&1 || { echo LB_FAIL $k; tail -30 $O/lb_kind$k.log; exit 1; }
echo "kind $k"; grep -E "fused A/B|mismatch|failed" $O/lb_kind$k.log | cut -c1-500
python3 -c "import json; d=json.loads([l for l in open('$O/lb_kind$k.log') if l.startswith('{')][-1]); c=d['config']; print('lb', d['ms_per_step'], c['fused_kernel'], min(c['stencil_variant_ms'].values()))"
done
