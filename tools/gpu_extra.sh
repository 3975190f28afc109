#!/bin/bash
# Secondary measurements for DESIGN.md: other BASELINE configs, NAT, host-memory path.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
        echo "rc($name)=$rc"; grep '^{' "gpurun_out/$name.log" | cut -c1-1500; if [ $rc -gt 1 ]; then exit $rc; fi; }
for w in ${WL:-c1 c3 c4}; do run bench_$w 300 python bench.py --workload $w --steps 100 --warmup 10 --cpu-budget 3; done
run natbench 200 python tools/natbench.py
run pattern_all 300 python tools/pattern_ceiling.py
# multi-rank control path rehearsed on one GPU (2 ranks share the card; the 8-GPU run is the driver's)
run bench_2rank 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 5
[ "${HOSTPATH:-0}" = 1 ] && run hostpath 400 python tools/hostpath.py
[ "${HOSTPATH:-0}" = 1 ] && { timeout -k 10 200 ./tools/flush_latency 2000 > gpurun_out/flush_latency.json 2> gpurun_out/flush_latency.err; echo "rc(flush_latency)=$?"; }
