#!/bin/bash
# One GPU-box pass, parameterised (replaces the per-experiment gpu_*.sh
# launchers of rounds 1-3). Usage, from the repo root on the box:
#
#   tools/gpu.sh NAME STEP [STEP ...]
#
# Output goes to gpurun_out/NAME/. Steps run in order, each under its own
# time limit; the pass stops at the first failure (no retries):
#
#   tests:F1,F2,...     pytest -m gpu on those files (-v -s, printed headroom logged)
#   suite               the whole -m gpu suite
#   smoke               __graft_entry__.smoke()
#   bench[:ARGS]        python bench.py ARGS            (bench.log / bench.json)
#   prof[:ARGS]         rocprofv3 --kernel-trace --stats over bench.py ARGS --no-cpu
#   torchrun[:ARGS]     bench.py through torch.distributed.run, 1 rank
#   py:SECS:SCRIPT ARGS python3 SCRIPT ARGS under a SECS limit (tools/*.py probes)
#   bin:SECS:BIN ARGS   a built probe binary (tools/dia_bench ...) under a SECS limit
#   pmc:SCRIPT          a tools/pmc_*.sh counter pass (each pass has its own limits)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
NAME=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$NAME
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
i=0
for step in "$@"; do
  i=$((i + 1))
  kind=${step%%:*}
  arg=""; [ "$kind" != "$step" ] && arg=${step#*:}
  log=$OUT/$(printf %02d $i)_$kind.log
  echo "== step $i: $step" | tee -a "$OUT/steps.log"
  case $kind in
    tests)
      timeout -k 10 900 python -u -m pytest --maxfail=8 -v -s --timeout 300 --timeout-method thread -m gpu ${arg//,/ } > "$log" 2>&1
      rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|headroom|max rel" "$log" | tail -60 ;;
    suite)
      timeout -k 10 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$log" 2>&1
      rc=$?; grep -E "Error|assert|FAILED" "$log" | head -20; tail -2 "$log" ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1
      rc=$?; tail -2 "$log" ;;
    bench)
      timeout -k 10 900 python bench.py $arg > "$log" 2>&1
      rc=$?; tail -1 "$log" > "$OUT/bench_$i.json"; tail -c 1500 "$log"; echo ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/prof_$i" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" $arg --no-cpu > "$log" 2>&1)
      rc=$?; tail -c 600 "$log"; echo ;;
    torchrun)
      timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus 1 $arg > "$log" 2>&1
      rc=$?; tail -1 "$log" ;;
    py)
      secs=${arg%%:*}; rest=${arg#*:}
      timeout -k 10 "$secs" python3 -u $rest > "$log" 2>&1
      rc=$?; tail -40 "$log" ;;
    bin)
      secs=${arg%%:*}; rest=${arg#*:}
      timeout -k 10 "$secs" $rest > "$log" 2>&1
      rc=$?; tail -40 "$log" ;;
    pmc)
      bash "$arg" > "$log" 2>&1
      rc=$?; tail -40 "$log" ;;
    *)
      echo "unknown step '$step'"; exit 2 ;;
  esac
  echo "== step $i rc=$rc" | tee -a "$OUT/steps.log"
  [ $rc -ne 0 ] && { tail -30 "$log"; exit $rc; }
done
exit 0
