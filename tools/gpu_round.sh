#!/bin/bash
# GPU-box sequence: parity tests -> short bench -> rocprofv3 kernel trace.  Every GPU step has
# its own time limit; a crash / abort / timeout (exit >1) ends the script immediately.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name" ; date +%T
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc($name)=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 400 python bench.py --steps 200 --warmup 20
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline
fi
