# Re-run the GPU test files up to test_gpu_halo.py once (order as in the full run).
O=gpurun_out/dbg; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_acoustic.py tests/test_checkpoint.py tests/test_examples.py tests/test_fused.py tests/test_gather.py tests/test_gpu_halo.py > $O/seq.log 2>&1; rc=$?
echo "rc=$rc"; tail -3 $O/seq.log; grep -A3 "AssertionError" $O/seq.log | head -20
