# Per-wave class timing of the fused kernel (tilings 40, 0; rounds 2; modes 0/1).
set -o pipefail
O=gpurun_out/waves; mkdir -p $O
timeout -k 10 300 python benchmarks/fused_waves.py --variants 40,0 --rounds 2 --mode 0 > $O/waves_m0.log 2>&1 || { echo W_FAIL; tail -20 $O/waves_m0.log; exit 1; }
grep -v amdgpu.ids $O/waves_m0.log
timeout -k 10 300 python benchmarks/fused_waves.py --variants 40 --rounds 2 --mode 1 > $O/waves_m1.log 2>&1 || { echo W_FAIL; tail -20 $O/waves_m1.log; exit 1; }
grep -v amdgpu.ids $O/waves_m1.log
