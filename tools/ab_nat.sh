#!/bin/bash
# A/B of two builds of libvpcsum.so on NAT (tooling): the tree's library ("new") against
# vproxy_amd/libvpcsum_ab.so ("old"), alternated per round; tools/natbench.py on the 10M C5 packets.
#   bash tools/ab_nat.sh [rounds]      writes gpurun_out/abnat_<new|old>_<round>.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
R=${1:-2}
cp vproxy_amd/libvpcsum.so /tmp/ab_new.so && cp vproxy_amd/libvpcsum_ab.so /tmp/ab_old.so || exit 1
for r in $(seq 1 "$R"); do
  for v in new old; do
    cp /tmp/ab_$v.so vproxy_amd/libvpcsum.so
    timeout -k 10 200 python tools/natbench.py 10000000 --no-cpu > "gpurun_out/abnat_${v}_$r.json" 2>&1 \
      || { cp /tmp/ab_new.so vproxy_amd/libvpcsum.so; exit 1; }
  done
done
cp /tmp/ab_new.so vproxy_amd/libvpcsum.so
for v in new old; do for r in $(seq 1 "$R"); do echo "$v $r: $(tail -1 gpurun_out/abnat_${v}_$r.json)"; done; done
