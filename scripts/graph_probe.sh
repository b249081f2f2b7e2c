mkdir -p gpurun_out/gp
run() { name=$1; shift; echo "== $name"; timeout -k 5 90 python benchmarks/graph_probe.py "$@" > gpurun_out/gp/$name.log 2>&1; rc=$?; cat gpurun_out/gp/$name.log | grep -v amdgpu.ids | grep -v "^[A-Z][a-z]* *[a-z]* *:"; echo "rc=$rc"; return $rc; }
run lb_seq loopback --mode sequential && run lb_one loopback --mode onephase && run lb_seq512 loopback --mode sequential --n 512 --steps 100
