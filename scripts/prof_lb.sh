set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
for m in sequential onephase; do
  IGG_HALO_MODE=$m timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_lb_$m -o run -- python3 $R/bench.py --loopback --periodic --graph --steps 50 --warmup 5 > $R/gpurun_out/prof_lb_$m.log 2>&1
  grep metric $R/gpurun_out/prof_lb_$m.log | cut -c1-300
done
