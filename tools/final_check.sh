#!/bin/bash
# Last check of a round's tree on one GPU (tooling): the GPU tests, smoke(), and the driver's own
# bench command three times.  usage: tools/final_check.sh <tag>; writes gpurun_out/<tag>_*
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=$1
python -c "import json; from vproxy_amd.build import source_hash; print(json.dumps({'src_hash': source_hash()}))" > gpurun_out/${TAG}_src.json || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 || { tail -20 gpurun_out/${TAG}_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_gputest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_driver_cmd_$i.log 2>&1 || exit 1
done
echo ALLDONE
