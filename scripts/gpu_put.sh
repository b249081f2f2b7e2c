R=$PWD
mkdir -p $R/gpurun_out/tr
cd /tmp && export TMPDIR=/tmp
for cu in 0 32; do
IGG_TRANSPORT=put timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr/cu$cu -o run -- python3 $R/benchmarks/trace_step.py --ir 0 --hv 11 --hr 0 --cu $cu > $R/gpurun_out/tr/cu$cu.log 2>&1
echo cu$cu rc=$?
done
