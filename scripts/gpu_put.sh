mkdir -p gpurun_out/put
timeout -k 10 500 python -m pytest tests/test_multiprocess.py tests/test_gpu_halo.py -x -v -k "put" > gpurun_out/put/mp.log 2>&1 || { tail -60 gpurun_out/put/mp.log; exit 1; }
tail -10 gpurun_out/put/mp.log
