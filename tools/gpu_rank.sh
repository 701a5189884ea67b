set -e
O=gpurun_out/rank; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_api.py -k hessian_reuse -x -q --timeout 200 --timeout-method thread > $O/test.log 2>&1
timeout -k 10 300 python tools/rank_sim.py --world 8 --rank 2 > $O/r2of8.log 2>&1
timeout -k 10 300 python tools/rank_sim.py --world 8 --all > $O/all8.log 2>&1
timeout -k 10 300 python tools/rank_sim.py --world 2 --all > $O/all2.log 2>&1
timeout -k 10 300 python tools/rank_sim.py --world 4 --all > $O/all4.log 2>&1
