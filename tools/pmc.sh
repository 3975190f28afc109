#!/bin/bash
# PMC passes (each its own rocprofv3 run, --pmc only, no sys/runtime/memory traces).
# usage: tools/pmc.sh "<prof_one.py args>" "CTR1 CTR2" "CTR3" ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; OUT=${OUT:-gpurun_out/pmc}; mkdir -p $OUT
ARGS="$1"; shift
i=0
for CTR in "$@"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $CTR --output-format csv -d $OUT -o p$i -- python3 tools/prof_one.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($CTR) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
