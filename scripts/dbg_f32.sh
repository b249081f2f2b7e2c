# Bisect the f32 NaN of test_gpu_diffusion_matches_reference (isolated vs after other tests).
O=gpurun_out/dbg; mkdir -p $O
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 200 $P tests/test_gpu_halo.py -k diffusion_matches > $O/alone.log 2>&1; rc=$?; echo "alone rc=$rc"; ok $rc || exit 1
timeout -k 10 300 $P tests/test_checkpoint.py tests/test_gpu_halo.py -k "restart or diffusion_matches" > $O/ckpt.log 2>&1; rc=$?; echo "ckpt+ rc=$rc"; ok $rc || exit 1
timeout -k 10 400 $P tests/test_fused.py tests/test_gpu_halo.py -k "fused or diffusion_matches" > $O/fused.log 2>&1; rc=$?; echo "fused+ rc=$rc"; ok $rc || exit 1
timeout -k 10 200 python -u scripts/dbg_f32.py > $O/f32.log 2>&1; rc=$?; echo "script rc=$rc"; grep -E "variant|BAD" $O/f32.log
