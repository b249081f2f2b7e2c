# Host AddressSanitizer run of the CPU test suite (GPU ASan is not available on the pool).
# Builds an ASan-instrumented copy of the tree in /tmp (the in-tree optimised .so that
# ships to the GPU box is left alone) and runs `pytest -m "not gpu"` with the clang ASan
# runtime preloaded (python itself is not instrumented). Multi-rank tests inherit it.
set -eo pipefail
D=${1:-/tmp/igg_asan}
rm -rf "$D" && mkdir -p "$D"
tar --exclude=.git --exclude=gpurun_out --exclude=build --exclude='*.so' -cf - . | tar -xf - -C "$D"
cd "$D" && python build.py --asan
nm -D implicitglobalgrid.jl_amd/_igg_native*.so | grep -q __asan_report || { echo "not instrumented"; exit 1; }
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 \
LD_PRELOAD=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1) \
IGG_AUTOBUILD=0 python -m pytest tests/ -q -m "not gpu" -p no:cacheprovider
