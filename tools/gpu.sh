#!/bin/bash
# The GPU calls of this repository as parameterised steps (round 4; the one-off scripts of
# rounds 1-3 are archived in tools/history/gpu_calls.md).  Run on the GPU box through gpurun:
#
#   gpurun -- 'bash tools/gpu.sh <tag> <step> [<step> ...]'
#
# Every step runs under its own time limit and writes under gpurun_out/<tag>/; the first step
# that fails, times out or faults ends the call (nothing else touches the GPU after it).
# In ARGS a '+' stands for a space (bench:c2:--steps+20+--warmup+5).  KEEP_GOING=1: a step that
# fails a check (rc 1: a red test) does not end the call; a time limit or a fault still does.
#
#   smoke                        __graft_entry__.smoke()
#   tests[:EXPR]                 the -m gpu suite (pytest -k EXPR), verbose, per-test timeout
#   bench:CFG[:ARGS]             python bench.py --config CFG ARGS -> bench_CFG.json
#   trace:CFG[:ARGS]             rocprofv3 --kernel-trace --stats of that bench -> trace_CFG/
#   pmc:CFG:CTRS[:ARGS]          one rocprofv3 --pmc pass (CTRS comma-separated) -> pmc_CFG_<n>/
#   ab:CFG:REPS:LIB[:ARGS]       REPS alternations: product library, then MPA_LIB=LIB (A/B on one box)
#   abenv:CFG:REPS:VAR=VAL[:ARGS] REPS alternations: default environment, then VAR=VAL
#   var:NAME:CFG:V=X,V=Y[:ARGS]  python bench.py --config CFG ARGS under V=X V=Y -> var_NAME.log
#   py:SCRIPT[:ARGS]             python tools/SCRIPT ARGS -> SCRIPT.log
#   probe:BIN[:ARGS]             tools/bin/BIN ARGS -> BIN.txt
set -u
TAG=${1:?usage: tools/gpu.sh TAG STEP...}
shift
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp

json_of() {  # the bench's JSON line
  grep '^{' "$1" > "$2" && python3 -c "import json,sys;d=json.load(open('$2'));r=d.get('roofline') or {};print('   ', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'kernel ms', r.get('avg_launch_ms'), 'frac', r.get('frac'), 'launches', r.get('launches'))"
}

run_step() {
  local step=$1
  IFS=':' read -r kind a b c d <<< "$step"
  a=${a:-}; b=${b:-}; c=${c:-}; d=${d:-}
  echo "== $step"
  case "$kind" in
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { r=$?; tail -20 "$O/smoke.log"; return $r; }
      tail -1 "$O/smoke.log" ;;
    tests)
      local k=()
      [ -n "$a" ] && k=(-k "${a//+/ }")
      timeout -k 10 1500 python -u -m pytest tests -m gpu -v -rP --timeout 240 --timeout-method thread "${k[@]}" > "$O/tests${TESTS_TAG:-}.log" 2>&1
      local rc=$?
      grep -E "^(FAILED|ERROR)|passed|failed" "$O/tests${TESTS_TAG:-}.log" | tail -5
      return $rc ;;
    bench)
      timeout -k 10 600 python -u bench.py --config "$a" ${b//+/ } > "$O/bench_$a.log" 2>&1 || { r=$?; tail -20 "$O/bench_$a.log"; return $r; }
      json_of "$O/bench_$a.log" "$O/bench_$a.json" ;;
    trace)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$a" -o "$a" -- python3 "$R/bench.py" --config "$a" --no-cpu-baseline ${b//+/ } > "$O/trace_$a.log" 2>&1) || { r=$?; tail -20 "$O/trace_$a.log"; return $r; }
      json_of "$O/trace_$a.log" "$O/trace_$a.json" ;;
    pmc)
      local n
      n=$(ls -d "$O"/pmc_"$a"_* 2>/dev/null | wc -l)
      (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${b//,/ } --output-format csv -d "$O/pmc_${a}_$n" -o "$a" -- python3 "$R/bench.py" --config "$a" --no-cpu-baseline ${c//+/ } > "$O/pmc_${a}_$n.log" 2>&1) || { r=$?; tail -20 "$O/pmc_${a}_$n.log"; return $r; }
      echo "    pmc pass $n ok" ;;
    ab)
      local i
      for i in $(seq 1 "$b"); do
        timeout -k 10 600 python -u bench.py --config "$a" --no-cpu-baseline ${d//+/ } > "$O/ab_${a}_A$i.log" 2>&1 || { r=$?; tail -20 "$O/ab_${a}_A$i.log"; return $r; }
        echo "  A $i $(grep '^{' "$O/ab_${a}_A$i.log" | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('avg_launch_ms'))")"
        MPA_LIB="$c" timeout -k 10 600 python -u bench.py --config "$a" --no-cpu-baseline ${d//+/ } > "$O/ab_${a}_B$i.log" 2>&1 || { r=$?; tail -20 "$O/ab_${a}_B$i.log"; return $r; }
        echo "  B $i $(grep '^{' "$O/ab_${a}_B$i.log" | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('avg_launch_ms'))")"
      done ;;
    abenv)
      local i
      for i in $(seq 1 "$b"); do
        timeout -k 10 600 python -u bench.py --config "$a" --no-cpu-baseline ${d//+/ } > "$O/abenv_${a}_A$i.log" 2>&1 || { r=$?; tail -20 "$O/abenv_${a}_A$i.log"; return $r; }
        echo "  A $i $(grep '^{' "$O/abenv_${a}_A$i.log" | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('avg_launch_ms'), (d.get('roofline') or {}).get('frac'))")"
        env "$c" timeout -k 10 600 python -u bench.py --config "$a" --no-cpu-baseline ${d//+/ } > "$O/abenv_${a}_B$i.log" 2>&1 || { r=$?; tail -20 "$O/abenv_${a}_B$i.log"; return $r; }
        echo "  B $i $(grep '^{' "$O/abenv_${a}_B$i.log" | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('avg_launch_ms'), (d.get('roofline') or {}).get('frac'))")"
      done ;;
    var)
      # var:NAME:CFG:VAR=VAL,VAR=VAL[:ARGS]  one bench under extra environment -> var_NAME.log
      local envs=()
      if [[ "$c" != *=* ]]; then  # no environment given: var:NAME:CFG:ARGS
        d=$c; c=
      fi
      IFS=',' read -r -a envs <<< "$c"
      env ${envs[@]+"${envs[@]}"} timeout -k 10 600 python -u bench.py --config "$b" --no-cpu-baseline ${d//+/ } > "$O/var_$a.log" 2>&1 || { r=$?; tail -20 "$O/var_$a.log"; return $r; }
      echo "  $a $(grep '^{' "$O/var_$a.log" | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('avg_launch_ms'), (d.get('roofline') or {}).get('frac'))")" ;;
    py)
      timeout -k 10 600 python -u "tools/$a" ${b//+/ } > "$O/${a%.py}.log" 2>&1 || { r=$?; tail -20 "$O/${a%.py}.log"; return $r; }
      tail -5 "$O/${a%.py}.log" ;;
    probe)
      timeout -k 10 300 "tools/bin/$a" ${b//+/ } > "$O/$a.txt" 2>&1 || { r=$?; tail -20 "$O/$a.txt"; return $r; }
      tail -5 "$O/$a.txt" ;;
    *)
      echo "unknown step $step"; return 2 ;;
  esac
}

# a failing step's exit status is the call's (124 / 137: its time limit; 134 / 139: an abort /
# a fault): nothing else runs after it
for s in "$@"; do
  run_step "$s"
  rc=$?
  if [ $rc -eq 1 ] && [ -n "${KEEP_GOING:-}" ]; then  # a failed check, not a limit or fault
    echo "step $s failed (rc 1): KEEP_GOING"
    continue
  fi
  if [ $rc -ne 0 ]; then
    echo "step $s failed (rc $rc): stopping"
    exit $rc
  fi
done
echo "all steps ok"
