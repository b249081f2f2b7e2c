# Lane-distributed z-segment edge loads (FEAT 512, variants 36-39): stencil GPU tests, then
# the interleaved variant x rounds sweep against their per-lane-load tilings.
set -o pipefail
O=gpurun_out/zl; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stencil.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_stencil.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error" $O/pytest_stencil.log | head; tail -30 $O/pytest_stencil.log; exit 1; }
tail -1 $O/pytest_stencil.log
timeout -k 10 400 python -u benchmarks/variant_sweep.py --variants 24,36,40,26,38 --rounds 1,2,3,4 > $O/variant_sweep.log 2>&1 || { echo SWEEP_FAIL; tail -20 $O/variant_sweep.log; exit 1; }
grep -v amdgpu.ids $O/variant_sweep.log | head -30
