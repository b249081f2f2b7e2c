mkdir -p gpurun_out/cfg
timeout -k 10 300 python -m pytest tests/test_acoustic.py -x -q > gpurun_out/cfg/pytest_acoustic.log 2>&1 || { tail -30 gpurun_out/cfg/pytest_acoustic.log; exit 1; }
tail -1 gpurun_out/cfg/pytest_acoustic.log
for c in acoustic2d diffusion3d_f32_gather; do
timeout -k 10 300 python bench.py --config $c --steps 200 --warmup 10 > gpurun_out/cfg/$c.log 2>&1 || { tail -20 gpurun_out/cfg/$c.log; exit 1; }
tail -1 gpurun_out/cfg/$c.log | cut -c1-900
done
timeout -k 10 300 python bench.py --config acoustic2d --steps 200 --warmup 10 --loopback --transport put > gpurun_out/cfg/acoustic_lb.log 2>&1 || { tail -20 gpurun_out/cfg/acoustic_lb.log; exit 1; }
tail -1 gpurun_out/cfg/acoustic_lb.log | cut -c1-400
