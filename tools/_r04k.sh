set -o pipefail; mkdir -p gpurun_out
python -c "import json,sys; sys.path.insert(0,'.'); from vproxy_amd.build import source_hash; json.dump({'src_hash': source_hash()}, open('gpurun_out/r04k_src.json','w'))" &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04k_gputest.log 2>&1 && tail -2 gpurun_out/r04k_gputest.log &&
timeout -k 10 900 bash tools/ab_libs_cold.sh r04k_ab "c3 c2 c4 c1" 2 "0 1" > gpurun_out/r04k_ab.log 2>&1; cat gpurun_out/r04k_ab.log
