#!/bin/bash
# A/B of two builds of libvpcsum.so on uncached (rotating) batches (tooling): the tree's library
# ("new") against vproxy_amd/libvpcsum_ab.so ("old"), alternated per round so that drift on the box
# hits both alike; compute and verify mode.  tools/cold_ab.py does the timing.
#   bash tools/ab_libs_cold.sh <tag> "<workloads>" [rounds] [modes]
# writes gpurun_out/<tag>_<new|old>_<w>_m<mode>_<round>.log and prints the medians
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=$1; WS=${2:-"c1 c3 c2"}; R=${3:-2}; MODES=${4:-"0 1"}
cp vproxy_amd/libvpcsum.so /tmp/ab_new.so && cp vproxy_amd/libvpcsum_ab.so /tmp/ab_old.so || exit 1
nb() { case $1 in c1) echo 16;; *) echo 2;; esac; }
for r in $(seq 1 "$R"); do
  for v in new old; do
    cp /tmp/ab_$v.so vproxy_amd/libvpcsum.so
    for w in $WS; do for m in $MODES; do
      timeout -k 10 150 python tools/cold_ab.py --workload "$w" --teams 0 --mode "$m" --batches "$(nb $w)" --rounds 2 \
        > "gpurun_out/${TAG}_${v}_${w}_m${m}_$r.log" 2>&1 || { cp /tmp/ab_new.so vproxy_amd/libvpcsum.so; exit 1; }
    done; done
  done
done
cp /tmp/ab_new.so vproxy_amd/libvpcsum.so
for w in $WS; do for m in $MODES; do for v in new old; do
  echo "$v $w mode $m: $(grep -h 'rotate' gpurun_out/${TAG}_${v}_${w}_m${m}_*.log | awk '{print $5}' | tr '\n' ' ')"
done; done; done
