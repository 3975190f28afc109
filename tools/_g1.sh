for w in c2 c3; do timeout -k 10 300 python tools/sweep.py --workload $w --teams 0,54,64,65 --bpc 2,4,5,8,12,16 --nt 1 --noout 2 --rounds 2 || exit 1; done
