set -o pipefail; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04q_gputest.log 2>&1 && tail -2 gpurun_out/r04q_gputest.log &&
timeout -k 10 600 bash tools/ab_libs_cold.sh r04q_ab "c1" 3 "1 0" > gpurun_out/r04q_ab.log 2>&1 && cat gpurun_out/r04q_ab.log &&
timeout -k 10 400 python tools/big_arena.py > gpurun_out/r04q_bigarena.log 2>&1; tail -c 1500 gpurun_out/r04q_bigarena.log
