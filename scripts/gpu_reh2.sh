mkdir -p gpurun_out/reh2
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/reh2/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/reh2/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/reh2/pytest_gpu.log
for np in 2 4; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port 2961$np bench.py --gpus $np --steps 50 --warmup 5 --local-n 256 --share-gpu > gpurun_out/reh2/b$np.log 2>&1 || { tail -30 gpurun_out/reh2/b$np.log; exit 1; }
grep "A/B" gpurun_out/reh2/b$np.log; grep -o '"ms_per_step": [0-9.]*\|"overlap_comm": [a-z]*\|"transport": "[a-z-]*"' gpurun_out/reh2/b$np.log | tr '\n' ' '; echo
done
