#!/bin/bash
# Verify against compute on uncached batches (tooling): compute (out words), verify with out words
# and status bytes, verify with status bytes only (the ingress result), alternated per round.
#   bash tools/verify_modes.sh <tag> "<workloads>" [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=$1; WS=${2:-"c1 c3 c2"}; R=${3:-3}
nb() { case $1 in c1) echo 16;; *) echo 2;; esac; }
for r in $(seq 1 "$R"); do
  for w in $WS; do
    timeout -k 10 150 python tools/cold_ab.py --workload $w --teams 0 --mode 0 --batches $(nb $w) --rounds 2 > gpurun_out/${TAG}_${w}_compute_$r.log 2>&1 || exit 1
    timeout -k 10 150 python tools/cold_ab.py --workload $w --teams 0 --mode 1 --batches $(nb $w) --rounds 2 > gpurun_out/${TAG}_${w}_verify_$r.log 2>&1 || exit 1
    timeout -k 10 150 python tools/cold_ab.py --workload $w --teams 0 --mode 1 --no-out --batches $(nb $w) --rounds 2 > gpurun_out/${TAG}_${w}_verifyst_$r.log 2>&1 || exit 1
  done
done
for w in $WS; do for k in compute verify verifyst; do
  echo "$w $k: $(grep -h 'rotate' gpurun_out/${TAG}_${w}_${k}_*.log | awk '{print $5}' | tr '\n' ' ')"
done; done
