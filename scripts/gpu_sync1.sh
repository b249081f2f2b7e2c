# Sync kernel with one release fence + relaxed polling: put/fused GPU tests, multi-rank put/fused, trace.
set -o pipefail
O=gpurun_out/sync1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -k "put or fused or loopback or multirank or gather or overlap" --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --loopback --periodic-dims xy --steps 60 --warmup 10 --fused on > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $R/$O/prof.log; exit 1; }
python3 $R/tools/trace_steps.py $R/$O/prof/run_kernel_trace.csv --main diffusion3d_hx --steps 30 --skip-last 12
