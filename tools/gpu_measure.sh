#!/bin/bash
# Measurement call (rounds 4-5): GPU tests, bench lines of every config, kernel traces, PMC passes
# (C2, C1, C3, C4, NAT full / read-only / pattern probe, the pre-image flush and its probe), host
# path.  Every GPU step has its own time limit; a crash / abort / timeout (exit > 1) ends the
# script.  usage: tools/gpu_measure.sh <tag> [parts]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04}; PARTS=${2:-tests,bench,trace,pmc,host}
step() {  # name, limit, cmd...
  local name=$1 lim=$2; shift 2
  echo "=== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "rc($name)=$rc"; tail -n 2 "gpurun_out/${TAG}_$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
has() { [[ ",$PARTS," == *",$1,"* ]]; }
# the measured tree: the hash of the library sources on this box (tools/save_profiles.py stores it
# in every summary.json; bench.py matches PMC summaries against it)
python -c "import json; from vproxy_amd.build import source_hash; print(json.dumps({'src_hash': source_hash()}))" > gpurun_out/${TAG}_src.json || exit 1
if has tests; then
  step gputest 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
fi
if has smoke; then
  step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
fi
if has benchc2; then
  step bench_c2 300 python bench.py --steps 200 --warmup 20
  step bench_c5 400 python bench.py --workload c5 --steps 50 --warmup 5
fi
if has bench; then
  step bench_c2 300 python bench.py --steps 200 --warmup 20
  for w in c1 c3 c4; do step bench_$w 300 python bench.py --workload $w --steps 200 --warmup 20; done
  step bench_c4_strong 300 python bench.py --workload c4 --strong --steps 200 --warmup 20 --no-cpu-baseline
  step bench_c5 400 python bench.py --workload c5 --steps 50 --warmup 5
  step bench_c5pre 400 python bench.py --workload c5 --preimage --steps 50 --warmup 5
fi
if has trace; then
  step trace_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline
fi
if has pmc || has pmck2; then   # pmck2: the checksum configs only (PMC_CFGS, default all four)
  # FETCH_SIZE takes 3 of the 4 TCC counters and WRITE_SIZE 2: never in one pass
  P="FETCH_SIZE|WRITE_SIZE|SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES|SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES|GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
  for w in ${PMC_CFGS:-c2 c1 c3 c4}; do
    IFS='|' read -ra PS <<< "$P"; i=0
    for c in "${PS[@]}"; do i=$((i+1)); step pmc_${w}_p$i 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_pmc_$w -o p$i -- python3 tools/prof_one.py --workload $w; done
  done
fi
if has pmc || has pmcnat; then
  N="FETCH_SIZE|WRITE_SIZE|TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum|SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
  for m in ${NAT_MASKS:-15 0}; do
    IFS='|' read -ra PS <<< "$N"; i=0
    for c in "${PS[@]}"; do i=$((i+1)); step pmc_nat${m}_p$i 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_pmc_nat$m -o p$i -- python3 tools/prof_one.py --nat 0 --nat-mask $m; done
  done
fi
if has pmc || has pmcnat || has pmcnatprobe; then   # NAT's memory operations without the rewrite
  N="FETCH_SIZE|WRITE_SIZE|TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"
  IFS='|' read -ra PS <<< "$N"; i=0
  for c in "${PS[@]}"; do i=$((i+1)); step pmc_natprobe_p$i 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_pmc_natprobe -o p$i -- python3 tools/prof_one.py --nat 0 --nat-mask 15 --nat-probe; done
  step trace_natprobe 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace_nat -o run -- python3 tools/prof_one.py --nat 0 --nat-mask 15 --nat-probe --iters 20
fi
if has pmc || has pmcpre; then   # the pre-image egress flush on C5 (bench --preimage's step) and its probe
  N="FETCH_SIZE|WRITE_SIZE|TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum|SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
  IFS='|' read -ra PS <<< "$N"; i=0
  for c in "${PS[@]}"; do i=$((i+1)); step pmc_pre15_p$i 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_pmc_pre15 -o p$i -- python3 tools/prof_one.py --pre 0; done
  i=0
  for c in FETCH_SIZE WRITE_SIZE; do i=$((i+1)); step pmc_preprobe_p$i 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_pmc_preprobe -o p$i -- python3 tools/prof_one.py --pre 0x800000; done
  step trace_c5pre 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace_c5pre -o run -- python3 bench.py --workload c5 --preimage --steps 50 --warmup 5 --no-cpu-baseline
fi
if has benchpre; then
  step bench_c5pre 400 python bench.py --workload c5 --preimage --steps 50 --warmup 5
fi
if has pmc32; then   # last: a counter this gfx950 image may not have
  step pmc_nat15_p32 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/${TAG}_pmc_nat15 -o p32 -- python3 tools/prof_one.py --nat 0 --nat-mask 15
fi
if has host; then
  step hostpath 400 python tools/hostpath.py
fi
if has flush; then   # tools/flush_latency is built in-tree beforehand (g++ line in its header)
  step flush 300 ./tools/flush_latency 2000
fi
if has rank8; then   # 8 ranks on one card: the strong shards per rank, a functional rehearsal
  step bench_c4s_8rank 600 python bench.py --workload c4 --strong --gpus 8 --steps 50 --warmup 5 --share-gpu --ramp-ms 300
  step bench_c5_8rank 600 python bench.py --workload c5 --gpus 8 --steps 20 --warmup 3 --share-gpu --ramp-ms 300
fi
if has pmcmode; then   # compute vs verify counters of the default kernel (PMC_CFGS, default c1)
  M="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES|FETCH_SIZE|WRITE_SIZE|SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  for w in ${PMC_CFGS:-c1}; do for m in 0 1; do
    IFS='|' read -ra PS <<< "$M"; i=0
    for c in "${PS[@]}"; do i=$((i+1)); step pmcm_${w}_m${m}_p$i 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_pmcm_${w}_m$m -o p$i -- python3 tools/prof_one.py --workload $w --mode $m; done
  done; done
fi
if has natrec; then   # two-stream NAT vs 32-B records, and their probes, one process, interleaved
  step natrec 600 python tools/natsweep.py --rec --rounds 4
fi
if has bigarena; then   # arenas past 4 GiB: windowed K2 vs views under 4 GiB vs the team kernel
  step bigarena 600 python tools/big_arena.py
fi
if has ab; then   # this tree's library against vproxy_amd/libvpcsum_ab.so, uncached batches, compute + verify
  step ab 1100 bash tools/ab_libs_cold.sh ${TAG}_ab "${AB_WS:-c1 c3 c2}" ${AB_ROUNDS:-2} "${AB_MODES:-0 1}"
fi
if has rank2; then   # the multi-rank path rehearsed on one GPU (bench.py launches its own ranks)
  step bench_c2_2rank 300 python bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline --share-gpu
  step bench_c5_2rank 400 python bench.py --workload c5 --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline --share-gpu
fi
if has preflush; then   # the NAT'd 1024-frame host flush, pre-image vs full recompute
  step preflush 300 python tools/preflush.py
fi
if has c3split; then   # C3 per size class: K2, unsorted, verify, grid / unit-order probes
  step c3split 300 python tools/c3_split.py
  step c3var 400 python tools/c3_variants.py --variants 0,79,78
fi
if has verify; then   # compute vs verify (out + status) vs status-only verify, uncached
  step verify 900 bash tools/verify_modes.sh ${TAG}_vm "c1 c3 c2" ${VM_ROUNDS:-2}
fi
echo ALLDONE
