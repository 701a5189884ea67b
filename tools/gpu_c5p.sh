set -e
O=gpurun_out/c5; mkdir -p $O
timeout -k 10 400 python -m cProfile -s cumtime tools/c5_probe.py --responses 64 --alphas 20 > $O/cprof.txt 2>&1
