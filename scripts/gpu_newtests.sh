set -o pipefail
O=gpurun_out/newtests; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py tests/test_multiprocess.py -m gpu -q -x -k "autotune or fused" --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
