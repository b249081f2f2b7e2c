mkdir -p gpurun_out/ac
timeout -k 10 300 python -m pytest tests/test_acoustic.py -x -q -m gpu > gpurun_out/ac/pytest.log 2>&1 || { tail -30 gpurun_out/ac/pytest.log; exit 1; }
tail -1 gpurun_out/ac/pytest.log
timeout -k 10 300 python bench.py --config acoustic2d --steps 200 --warmup 10 > gpurun_out/ac/bench.log 2>&1 || { tail -20 gpurun_out/ac/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"t_eff_per_gpu_GBs": [0-9.]*' gpurun_out/ac/bench.log
timeout -k 10 300 python bench.py --steps 200 --warmup 10 > gpurun_out/ac/bench3d.log 2>&1 || { tail -20 gpurun_out/ac/bench3d.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"t_eff_per_gpu_GBs": [0-9.]*\|"stencil_variant.*' gpurun_out/ac/bench3d.log
