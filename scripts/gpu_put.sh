mkdir -p gpurun_out/put2
timeout -k 10 500 python -m pytest tests -x -q -m gpu -k "put or loopback or acoustic" > gpurun_out/put2/pytest.log 2>&1 || { tail -40 gpurun_out/put2/pytest.log; exit 1; }
tail -1 gpurun_out/put2/pytest.log
IGG_TRANSPORT=put timeout -k 10 100 python benchmarks/halo_only.py --reps 50 2>&1 | grep halo_us
for g in "" "--no-graph"; do
timeout -k 10 180 python bench.py --steps 200 --warmup 20 --loopback --periodic --transport put $g > gpurun_out/put2/bench$g.log 2>&1 || { tail -20 gpurun_out/put2/bench$g.log; exit 1; }
echo "== put $g $(grep -o '"ms_per_step": [0-9.]*\|"phase_ms": {[^}]*}\|"stencil_variant": [0-9]*' gpurun_out/put2/bench$g.log | tr '\n' ' ')"
done
