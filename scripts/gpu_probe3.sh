# RCCL capture reproducer (phase markers) + fused cost grid (tiling 0 / 50) for arena kinds 3 and 1.
set -o pipefail
O=gpurun_out/probe3; mkdir -p $O
timeout -k 10 300 python benchmarks/rccl_capture_repro.py side_kern fork_join_first > $O/rccl_capture.log 2>&1; echo "repro rc=$?"
cat $O/rccl_capture.log
for k in 3 1; do
IGG_PUT_ARENA_KIND=$k timeout -k 10 300 python benchmarks/fused_sweep.py --grid --variants 0,50 > $O/fused_grid_kind$k.log 2>&1 || { echo GRID_FAIL; tail -20 $O/fused_grid_kind$k.log; exit 1; }
echo "kind $k"; grep -v amdgpu.ids $O/fused_grid_kind$k.log
done
