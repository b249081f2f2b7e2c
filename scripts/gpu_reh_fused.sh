# Rehearsal of the multi-rank bench flow on one GPU (ranks share device 0):
# transport A/B, fused check + A/B, graph capture, close, finalize.
set -o pipefail
mkdir -p gpurun_out/reh
for np in 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port 2961$np bench.py --gpus $np --steps 40 --warmup 4 --local-n 160 --share-gpu > gpurun_out/reh/f$np.log 2>&1 || { echo FAIL $np; tail -30 gpurun_out/reh/f$np.log; exit 1; }
  grep -E "A/B|^\{" gpurun_out/reh/f$np.log | cut -c1-420
done
