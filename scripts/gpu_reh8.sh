# 8-rank shared-GPU rehearsal: default HW queues vs GPU_MAX_HW_QUEUES=1 (queue oversubscription hypothesis).
set -o pipefail
O=gpurun_out/reh8; mkdir -p $O
for q in default 1; do
if [ $q = default ]; then
timeout -k 10 500 python bench.py --gpus 8 --share-gpu --n 160 --steps 50 --warmup 5 --launch-timeout 450 > $O/reh8_$q.log 2>&1 || { echo R_FAIL $q; tail -30 $O/reh8_$q.log; exit 1; }
else
GPU_MAX_HW_QUEUES=$q timeout -k 10 500 python bench.py --gpus 8 --share-gpu --n 160 --steps 50 --warmup 5 --launch-timeout 450 > $O/reh8_$q.log 2>&1 || { echo R_FAIL $q; tail -30 $O/reh8_$q.log; exit 1; }
fi
echo "== queues $q"; grep -E "A/B|validation" $O/reh8_$q.log | cut -c1-400; tail -1 $O/reh8_$q.log | cut -c1-200
done
