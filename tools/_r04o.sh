set -o pipefail; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04o_gputest.log 2>&1 && tail -2 gpurun_out/r04o_gputest.log &&
timeout -k 10 900 bash tools/ab_libs_cold.sh r04o_ab "c1 c3 c2" 2 "1 0" > gpurun_out/r04o_ab.log 2>&1; cat gpurun_out/r04o_ab.log
