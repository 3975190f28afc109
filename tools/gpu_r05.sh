#!/bin/bash
# Round-5 GPU steps (tooling): usage tools/gpu_r05.sh <tag> <step>...; every step under its own
# time limit, the first failure ends the call.  Logs and JSON lines under gpurun_out/<tag>_*.
#   pre       the pre-image GPU tests          gputest  every GPU test
#   bench     bench.py C2 (the driver's line)  c5pre    bench.py --workload c5 --preimage
#   c5        bench.py --workload c5 (NAT)     c3 / c1 / c4  bench.py --workload cN
#   smoke     __graft_entry__.smoke()
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=$1; shift
for step in "$@"; do
  case $step in
    pre) timeout -k 10 400 python -u -m pytest tests/test_gpu_pre.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pre.log 2>&1 || { tail -30 gpurun_out/${TAG}_pre.log; exit 1; }
         tail -1 gpurun_out/${TAG}_pre.log ;;
    gputest) timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -30 gpurun_out/${TAG}_gputest.log; exit 1; }
         tail -1 gpurun_out/${TAG}_gputest.log ;;
    smoke) timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
         tail -1 gpurun_out/${TAG}_smoke.log ;;
    bench) timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || { tail -5 gpurun_out/${TAG}_bench_c2.err; exit 1; } ;;
    c5pre) timeout -k 10 400 python3 bench.py --workload c5 --preimage --steps 50 --warmup 5 > gpurun_out/${TAG}_bench_c5pre.json 2> gpurun_out/${TAG}_bench_c5pre.err || { tail -5 gpurun_out/${TAG}_bench_c5pre.err; exit 1; } ;;
    c5) timeout -k 10 400 python3 bench.py --workload c5 --steps 50 --warmup 5 > gpurun_out/${TAG}_bench_c5.json 2> gpurun_out/${TAG}_bench_c5.err || { tail -5 gpurun_out/${TAG}_bench_c5.err; exit 1; } ;;
    c1|c3|c4) timeout -k 10 300 python3 bench.py --workload $step --steps 200 --warmup 20 > gpurun_out/${TAG}_bench_$step.json 2> gpurun_out/${TAG}_bench_$step.err || { tail -5 gpurun_out/${TAG}_bench_$step.err; exit 1; } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo ALLDONE
