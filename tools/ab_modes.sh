#!/bin/bash
# A/B of K2 tuning mode bits in one library on uncached (rotating) batches (tooling): each mode
# value in turn, alternated per round so that drift on the box hits all alike.  tools/cold_ab.py
# does the timing.
#   bash tools/ab_modes.sh <tag> "<workloads>" [rounds] "<modes>"
# writes gpurun_out/<tag>_<w>_m<mode>_<round>.log and prints the medians
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=$1; WS=${2:-"c3 c1 c2 c4"}; R=${3:-2}; MODES=${4:-"0 32768"}
nb() { case $1 in c1) echo 16;; *) echo 2;; esac; }
for r in $(seq 1 "$R"); do
  for w in $WS; do for m in $MODES; do
    timeout -k 10 150 python tools/cold_ab.py --workload "$w" --teams 0 --mode "$m" --batches "$(nb $w)" --rounds 2 \
      > "gpurun_out/${TAG}_${w}_m${m}_$r.log" 2>&1 || exit 1
  done; done
done
for w in $WS; do for m in $MODES; do
  echo "$w mode $m: $(grep -h 'rotate' gpurun_out/${TAG}_${w}_m${m}_*.log | awk '{print $5}' | tr '\n' ' ')"
done; done
