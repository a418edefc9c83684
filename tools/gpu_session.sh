#!/bin/bash
# One parametrised GPU-box runner (replaces the per-session tools/gpu_r0*.sh one-offs of rounds 3-5).
#
#   tools/gpu_session.sh TASK[:ARG] [TASK[:ARG] ...]      e.g. via gpurun:
#   gpurun --timeout 900 -- 'tools/gpu_session.sh tests smoke bench:3 "prof:base|--steps 5 --warmup 2"'
#
# Tasks (each under its own time limit; the session stops at the first failure, so nothing more runs on
# a GPU after a fault, an abort or a time-out):
#   tests[:K]              pytest -m gpu (optionally -k K), one process, per-test thread time-outs
#   smoke                  __graft_entry__.smoke()
#   bench[:N]              python bench.py $BENCH_ARGS, N times (default 1), JSON lines -> $O/bench.jsonl
#   run:NAME|ARGS          python bench.py ARGS -> $O/NAME.log (the JSON line also -> $O/bench.jsonl)
#   envrun:NAME|VAR=V ..|ARGS  the same with extra environment (e.g. DPA_LIB_PATH=build/ab/X/libdpa_hip.so)
#   prof:NAME|ARGS         rocprofv3 --kernel-trace --stats of bench.py ARGS -> $O/NAME/, summary NAME.txt
#   pmc:NAME|COUNTERS|ARGS rocprofv3 --pmc COUNTERS (one pass) of bench.py ARGS -> $O/NAME/
#   py:NAME|SCRIPT ARGS    python SCRIPT ARGS -> $O/NAME.log (tools that need the GPU)
# Environment: O (output dir, default gpurun_out/session), BENCH_ARGS, LIMIT (seconds per step, 600).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
R=$PWD
O=${O:-gpurun_out/session}
LIMIT=${LIMIT:-600}
mkdir -p "$O"

step() {  # name, then the command: run under a time limit, report, stop the session on failure
  local name=$1; shift
  local t0=$(date +%s)
  "$@"
  local rc=$?
  echo "[session] $name rc=$rc ($(( $(date +%s) - t0 )) s)"
  if [ $rc -ne 0 ]; then exit $rc; fi
}

for task in "$@"; do
  kind=${task%%:*}
  arg=${task#*:}; [ "$arg" = "$task" ] && arg=""
  case $kind in
    tests)
      step tests timeout -k 10 ${LIMIT_TESTS:-1200} python -u -m pytest tests -m gpu -x -q --timeout 300 \
        --timeout-method thread ${arg:+-k "$arg"} > "$O/pytest_gpu.log" 2>&1
      tail -2 "$O/pytest_gpu.log" ;;
    smoke)
      step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
      tail -1 "$O/smoke.log" ;;
    bench)
      for i in $(seq 1 ${arg:-1}); do
        step "bench$i" timeout -k 10 $LIMIT python bench.py $BENCH_ARGS --out "$O/bench.jsonl" > "$O/bench_$i.log" 2>&1
        tail -1 "$O/bench_$i.log" | cut -c1-220
      done ;;
    run)
      name=${arg%%|*}; args=${arg#*|}
      step "$name" timeout -k 10 $LIMIT python bench.py $args --out "$O/bench.jsonl" > "$O/$name.log" 2>&1
      tail -1 "$O/$name.log" | cut -c1-260 ;;
    envrun)
      name=${arg%%|*}; rest=${arg#*|}; vars=${rest%%|*}; args=${rest#*|}
      step "$name" env $vars timeout -k 10 $LIMIT python bench.py $args --out "$O/bench.jsonl" > "$O/$name.log" 2>&1
      tail -1 "$O/$name.log" | cut -c1-260 ;;
    prof)
      name=${arg%%|*}; args=${arg#*|}
      rm -rf "$O/$name"
      step "prof-$name" bash -c "cd /tmp && timeout -k 10 $LIMIT rocprofv3 --kernel-trace --stats --output-format csv \
        -d $R/$O/$name -o run -- python3 $R/bench.py $args > $R/$O/$name.log 2>&1"
      python tools/prof_summary.py "$O/$name" --timeline > "$O/$name.txt" 2>&1
      head -12 "$O/$name.txt" | cut -c1-130 ;;
    pmc)
      name=${arg%%|*}; rest=${arg#*|}; ctrs=${rest%%|*}; args=${rest#*|}
      rm -rf "$O/$name"
      step "pmc-$name" bash -c "cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv \
        -d $R/$O/$name -o run -- python3 $R/bench.py $args > $R/$O/$name.log 2>&1" ;;
    py)
      name=${arg%%|*}; cmd=${arg#*|}
      step "$name" timeout -k 10 $LIMIT python $cmd > "$O/$name.log" 2>&1
      tail -3 "$O/$name.log" | cut -c1-260 ;;
    *)
      echo "unknown task $kind"; exit 2 ;;
  esac
done
