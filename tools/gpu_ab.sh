#!/bin/bash
# A/B call: GPU tests, then kernel variants on rotating (uncached) batches and the bench lines.
# usage: tools/gpu_ab.sh <tag> "<c1 variants>" "<c3 variants>"   (every step has its own limit)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; V1=${2:-79,76,77}; V3=${3:-79,76}
run() { local name=$1 lim=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_$name.txt" 2>&1; local rc=$?; echo "rc($name)=$rc"; tail -n 12 "gpurun_out/${TAG}_$name.txt"; [ $rc -eq 0 ] || exit $rc; }
[ "${SKIP_TESTS:-0}" = 1 ] || run gputest 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run c1_ab 400 python tools/cold_ab.py --workload c1 --teams "$V1" --batches 16 --rounds 4
run c3_ab 400 python tools/cold_ab.py --workload c3 --teams "$V3" --batches 2 --rounds 3
run c2_ab 400 python tools/cold_ab.py --workload c2 --teams "$V3" --batches 2 --rounds 3
run bench_c1 300 python bench.py --workload c1 --steps 200 --warmup 20
run bench_c2 300 python bench.py --steps 200 --warmup 20
echo ALLDONE
