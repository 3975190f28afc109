timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; tail -3 gpurun_out/pytest_gpu.log
for w in c2 c3 c1 c4; do timeout -k 10 120 python tools/sweep.py --workload $w --teams 0,27,40,46,50,54 --bpc 0 --nt 1 --noout 2 || exit 1; done
