# Stream-ordered direct-pull gather_async_ + row reorder kernel: GPU suite, 2/4-rank shared-GPU gather bench.
set -o pipefail
O=gpurun_out/gather2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 170 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -m pytest tests/test_multiprocess.py -q -k gather --timeout 170 --timeout-method thread > $O/pytest_mp_gather.log 2>&1 || { echo MP_FAIL; tail -60 $O/pytest_mp_gather.log; exit 1; }
tail -1 $O/pytest_mp_gather.log
for n in 2 4; do
timeout -k 10 400 python bench.py --config diffusion3d_f32_gather --gpus $n --share-gpu --n 256 --steps 200 --warmup 5 --launch-timeout 350 > $O/bench_gather_$n.log 2>&1 || { echo B_FAIL $n; tail -30 $O/bench_gather_$n.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench_gather_$n.log') if l.startswith('{')][-1]); c=d['config']; print('$n ranks', d['ms_per_step'], 'gather_ms', c['gather_ms'], c['gather_mode'])"
done
