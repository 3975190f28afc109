set -o pipefail; mkdir -p gpurun_out
python -c "import json; from vproxy_amd.build import source_hash; print(json.dumps({'src_hash': source_hash()}))" > gpurun_out/r04p_src.json &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04p_smoke.log 2>&1 && tail -1 gpurun_out/r04p_smoke.log &&
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04p_driver_cmd_$i.log 2>&1 || exit 1; tail -c 300 gpurun_out/r04p_driver_cmd_$i.log; echo; done &&
timeout -k 10 300 python bench.py --gpus 2 --steps 50 --warmup 5 --share-gpu > gpurun_out/r04p_bench_c2_2rank.log 2>&1 && tail -c 300 gpurun_out/r04p_bench_c2_2rank.log
