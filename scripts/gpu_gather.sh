mkdir -p gpurun_out/ga
timeout -k 10 300 python -m pytest tests/test_multiprocess.py -x -q -k "gather" -m gpu > gpurun_out/ga/pytest.log 2>&1 || { tail -40 gpurun_out/ga/pytest.log; exit 1; }
tail -1 gpurun_out/ga/pytest.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29641 bench.py --gpus 2 --config diffusion3d_f32_gather --local-n 256 --steps 200 --warmup 4 --share-gpu --transport put > gpurun_out/ga/b2.log 2>&1 || { tail -30 gpurun_out/ga/b2.log; exit 1; }
grep metric gpurun_out/ga/b2.log | cut -c1-200; grep -o '"gather_ms": [0-9.]*\|"gather_mode": "[a-z]*"' gpurun_out/ga/b2.log
timeout -k 10 300 python bench.py --config diffusion3d_f32_gather --steps 200 --warmup 10 > gpurun_out/ga/b1.log 2>&1 || { tail -30 gpurun_out/ga/b1.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"gather_ms": [0-9.]*' gpurun_out/ga/b1.log
