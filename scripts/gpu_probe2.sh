# Paired strided-face pack probe + RCCL hipGraph capture reproducer.
set -o pipefail
O=gpurun_out/probe2; mkdir -p $O
timeout -k 10 120 python benchmarks/pack_faces.py > $O/pack_faces.log 2>&1 || { echo PACK_FAIL; tail -20 $O/pack_faces.log; exit 1; }
grep -v amdgpu.ids $O/pack_faces.log
timeout -k 10 700 python benchmarks/rccl_capture_repro.py > $O/rccl_capture.log 2>&1; echo "repro rc=$?"
cat $O/rccl_capture.log
