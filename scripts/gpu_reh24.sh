# Multi-rank bench rehearsal (2 and 4 ranks share device 0) + multi-rank fused GPU tests.
set -o pipefail
O=gpurun_out/reh24; mkdir -p $O
for np in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port 2962$np bench.py --gpus $np --steps 40 --warmup 4 --local-n 160 --share-gpu > $O/f$np.log 2>&1 || { echo FAIL $np; tail -30 $O/f$np.log; exit 1; }
  grep -E "A/B|^\{" $O/f$np.log | cut -c1-600
done
timeout -k 10 400 python -u -m pytest tests/test_multiprocess.py -m gpu -x -v -k fused --timeout 300 --timeout-method thread > $O/pytest_mp_fused.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_mp_fused.log; exit 1; }
tail -1 $O/pytest_mp_fused.log
