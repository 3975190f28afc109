#!/bin/bash
# rocprofv3 kernel traces (--kernel-trace --stats) of the bench command of each config, on the tree
# as it is (tooling).  usage: tools/trace_cfgs.sh <tag> [configs]; writes gpurun_out/<tag>_trace_<cfg>/
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; CFGS=${2:-"c1 c3 c4 c5"}
python -c "import json; from vproxy_amd.build import source_hash; print(json.dumps({'src_hash': source_hash()}))" > gpurun_out/${TAG}_src.json || exit 1
for w in $CFGS; do
  steps=200; warm=20; [ "$w" = c5 ] && { steps=50; warm=5; }
  echo "=== trace_$w $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace_$w -o run -- \
    python3 bench.py --workload $w --steps $steps --warmup $warm --no-cpu-baseline > gpurun_out/${TAG}_trace_$w.log 2>&1
  rc=$?; echo "rc(trace_$w)=$rc"; tail -c 400 gpurun_out/${TAG}_trace_$w.log; echo
  rm -f gpurun_out/${TAG}_trace_$w/run_kernel_trace.csv   # per-launch rows: tens of MB; the stats stay
  [ $rc -ne 0 ] && exit $rc
done
echo ALLDONE
