#!/bin/bash
# One parameterised GPU-box run (replaces the round's one-off scripts):
#   tools/gpu_round.sh OUTDIR STEP [STEP ...]
# writes under gpurun_out/OUTDIR.  Steps, run in the order given, each under its
# own time limit; the first failure ends the run (set -e), so a fault, abort or
# timeout starts nothing more on the GPU:
#   tests      pytest -m gpu (the whole GPU suite)
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py (the default bench line)
#   prof       tools/prof_round.sh OUTDIR: bench, bench under rocprofv3 --kernel-trace
#              --stats, FETCH_SIZE / WRITE_SIZE and SQ passes
#   sets       tools/bench_sets.py (share-set calls)
#   segment    tools/bench_segment.py (streamed upload)
#   lib=PATH   A/B: bench.py against another build of the library (--lib PATH)
#   batch=B    bench.py with B segments per launch (--batch B)
#   trace      a short bench.py under rocprofv3 --kernel-trace --stats (per-dispatch times)
#   py=SCRIPT  any other python script under tools/ (args after a colon: py=tools/x.py:--a:1)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1
shift
O=gpurun_out/$OUT
mkdir -p $O
for step in "$@"; do
  echo "[$(date +%T)] $step" >> $O/steps.log
  case $step in
    tests) timeout -k 10 900 python -u -m pytest -x -q --durations=25 --timeout 200 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 ;;
    bench) timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1 ;;
    prof) bash tools/prof_round.sh $OUT ;;
    sets) timeout -k 10 200 python -u tools/bench_sets.py > $O/bench_sets.json 2> $O/bench_sets.err ;;
    segment) timeout -k 10 200 python -u tools/bench_segment.py > $O/bench_segment.log 2>&1 ;;
    lib=*) timeout -k 10 500 python -u bench.py --lib ${step#lib=} --no-cpu-baseline --no-other-configs >> $O/bench_lib.log 2>&1 ;;
    batch=*) timeout -k 10 500 python -u bench.py --batch ${step#batch=} --no-cpu-baseline --no-other-configs >> $O/bench_batch.log 2>&1 ;;
    trace) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-other-configs > $O/bench_trace.log 2>&1 ;;
    py=*) spec=${step#py=}; IFS=: read -ra a <<< "$spec"
          timeout -k 10 600 python -u "${a[@]}" >> $O/$(basename ${a[0]} .py).log 2>&1 ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo all-done > $O/done
