mkdir -p gpurun_out/reh
timeout -k 10 200 python bench.py --steps 100 --warmup 10 > gpurun_out/reh/b1.log 2>&1 || { tail -20 gpurun_out/reh/b1.log; exit 1; }
tail -1 gpurun_out/reh/b1.log | cut -c1-400
for np in 2 8; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $np --steps 50 --warmup 5 --local-n 192 --share-gpu > gpurun_out/reh/b$np.log 2>&1 || { tail -30 gpurun_out/reh/b$np.log; exit 1; }
grep "transport A/B\|metric" gpurun_out/reh/b$np.log | cut -c1-300
done
