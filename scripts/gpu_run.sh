#!/bin/bash
# One parametrized runner for GPU-box measurements (replaces the per-run
# scripts of rounds 1-2, which stay in git history next to their profiles/).
#
# usage: scripts/gpu_run.sh TAG STEP [STEP ...]
#   Every STEP is one quoted argument: "[VAR=value ...] KIND[@SECONDS] [ARGS...]"
#   KIND  smoke                      __graft_entry__.smoke()
#         pytest  [pytest args]      python -u -m pytest -x -q --timeout 120 (-m gpu unless -m given;
#                                    --kor=a,b,c for -k "a or b or c")
#         bench   [bench.py args]    python bench.py ... (prints the JSON summary line)
#         py      script.py [args]   any python script of the repo
#         prof    [bench.py args]    rocprofv3 --kernel-trace --stats around bench.py
#         profpy  script.py [args]   the same around any python script of the repo
#         pmc     COUNTERS [bench.py args]   one rocprofv3 --pmc pass (COUNTERS comma-separated)
#         pmcpy   COUNTERS script.py [args]  the same around any python script of the repo
#   Logs go to gpurun_out/TAG/NN_KIND.log. Each step runs under its own
#   `timeout -k 10` (default per kind, or KIND@SECONDS); the first failing step
#   ends the script (no GPU step runs after a failure, a timeout or a fault).
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
i=0
for step in "$@"; do
  i=$((i + 1))
  read -r -a tok <<< "$step"
  envs=()
  while [[ ${tok[0]} == *=* && ${tok[0]} =~ ^[A-Z_][A-Z0-9_]*= ]]; do envs+=("${tok[0]}"); tok=("${tok[@]:1}"); done
  kind=${tok[0]}; args=("${tok[@]:1}")
  to=""
  if [[ $kind == *@* ]]; then to=${kind#*@}; kind=${kind%@*}; fi
  log=$(printf "%s/%02d_%s.log" "$O" "$i" "$kind")
  case $kind in
    smoke) to=${to:-240}; cmd=(python -u -c "import __graft_entry__ as g; g.smoke()") ;;
    pytest)
      to=${to:-900}
      marks=(-m gpu); for a in "${args[@]}"; do [[ $a == -m ]] && marks=(); done
      # --kor=a,b,c -> -k "a or b or c" (a step is split on whitespace)
      pargs=()
      for a in "${args[@]}"; do
        if [[ $a == --kor=* ]]; then k=${a#--kor=}; pargs+=(-k "${k//,/ or }"); else pargs+=("$a"); fi
      done
      cmd=(python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider "${marks[@]}" "${pargs[@]}") ;;
    bench) to=${to:-400}; cmd=(python -u bench.py "${args[@]}") ;;
    py) to=${to:-400}; cmd=(python -u "${args[@]}") ;;
    prof)
      to=${to:-300}
      cmd=(rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof$i" -o run -- python3 "$R/bench.py" "${args[@]}") ;;
    profpy)
      to=${to:-300}
      cmd=(rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof$i" -o run -- python3 "$R/${args[0]}" "${args[@]:1}") ;;
    pmcpy)
      to=${to:-120}
      cmd=(rocprofv3 --pmc "${args[0]//,/ }" --output-format csv -d "$O/pmc$i" -o run -- python3 "$R/${args[1]}" "${args[@]:2}") ;;
    pmc)
      to=${to:-120}
      cmd=(rocprofv3 --pmc "${args[0]//,/ }" --output-format csv -d "$O/pmc$i" -o run -- python3 "$R/bench.py" "${args[@]:1}") ;;
    *) echo "gpu_run: unknown step kind '$kind'"; exit 2 ;;
  esac
  echo "== [$i] ${envs[*]} $kind ${args[*]} (timeout $to s) -> $log"
  (
    for e in "${envs[@]}"; do export "$e"; done
    if [[ $kind == prof* || $kind == pmc* ]]; then cd /tmp || exit 1; fi
    timeout -k 10 "$to" "${cmd[@]}"
  ) > "$log" 2>&1
  rc=$?
  if [[ $kind == bench || $kind == prof ]]; then
    grep -E "A/B|validation|check" "$log" | cut -c1-400
    grep -E '^\{' "$log" | tail -1 | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); c = d['config']
    print('  ->', d['ms_per_step'], 'ms/step', d['value'], d['unit'], 'transport', c.get('transport'),
          'fused', c.get('fused_kernel'), 'post', c.get('post_validation'), c.get('fused_post_check'))" 2>/dev/null
  else
    tail -4 "$log"
  fi
  if [[ $rc -ne 0 ]]; then
    echo "== [$i] $kind FAILED rc=$rc"; tail -30 "$log"; exit 1
  fi
done
echo "== all $i steps ok"
