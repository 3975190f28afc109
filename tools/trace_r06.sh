#!/bin/bash
# Round 6 traces: rocprofv3 --kernel-trace --stats of the bench commands (c2 headline, c5 NAT
# production kernel, c5 pre-image flush), each in its own run.  usage: tools/trace_r06.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1
python -c "import json; from vproxy_amd.build import source_hash; print(json.dumps({'src_hash': source_hash()}))" > gpurun_out/${TAG}_src.json || exit 1
run() {   # name, bench args...
  local name=$1; shift
  echo "=== trace_$name $(date +%T)"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace_$name -o run -- \
    python3 bench.py "$@" --no-cpu-baseline > gpurun_out/${TAG}_trace_$name.log 2>&1
  local rc=$?; echo "rc(trace_$name)=$rc"; tail -c 300 gpurun_out/${TAG}_trace_$name.log; echo
  rm -f gpurun_out/${TAG}_trace_$name/run_kernel_trace.csv
  return $rc
}
run c2 --workload c2 --steps 200 --warmup 20 && \
run c5 --workload c5 --steps 50 --warmup 5 && \
run c5pre --workload c5 --preimage --steps 50 --warmup 5 && echo ALLDONE
