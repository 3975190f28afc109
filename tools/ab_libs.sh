#!/bin/bash
# A/B of two builds of libvpcsum.so on one box (tooling): the tree's library ("new") against
# vproxy_amd/libvpcsum_ab.so ("old"), alternated per round so that drift hits both alike.
#   bash tools/ab_libs.sh "<workloads>" [rounds] [extra sweep args]
# writes gpurun_out/ab_<new|old>_<w>_<round>.log (tools/sweep.py output)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
WS=${1:-"c2 c3 c4 c1"}; R=${2:-2}; shift 2 2>/dev/null
cp vproxy_amd/libvpcsum.so /tmp/ab_new.so && cp vproxy_amd/libvpcsum_ab.so /tmp/ab_old.so || exit 1
for r in $(seq 1 "$R"); do
  for v in new old; do
    cp /tmp/ab_$v.so vproxy_amd/libvpcsum.so
    for w in $WS; do
      timeout -k 10 120 python tools/sweep.py --workload "$w" --teams 0 --nt 1 --rounds 3 --iters 30 "$@" \
        > "gpurun_out/ab_${v}_${w}_$r.log" 2>&1 || { cp /tmp/ab_new.so vproxy_amd/libvpcsum.so; exit 1; }
    done
  done
done
cp /tmp/ab_new.so vproxy_amd/libvpcsum.so
for w in $WS; do for v in new old; do
  echo "$v $w: $(grep -h 'variant=' gpurun_out/ab_${v}_${w}_*.log | awk '{print $6}' | tr '\n' ' ')"
done; done
