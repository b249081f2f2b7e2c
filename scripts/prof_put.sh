set -e
R=$PWD
mkdir -p $R/gpurun_out/pp
IGG_TRANSPORT=put timeout -k 10 100 python benchmarks/halo_only.py --reps 50
IGG_TRANSPORT=put timeout -k 10 100 python benchmarks/halo_only.py --reps 50 --dims 1,0,0
timeout -k 10 100 python benchmarks/halo_only.py --reps 50
cd /tmp && export TMPDIR=/tmp
IGG_TRANSPORT=put timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pp/put -o run -- python3 $R/benchmarks/halo_only.py --reps 20 > $R/gpurun_out/pp/put.log 2>&1
