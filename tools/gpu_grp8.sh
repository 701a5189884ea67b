set -e
O=gpurun_out/grp8; mkdir -p $O
timeout -k 10 300 python tools/rank_sim.py --world 8 --all > $O/g1.log 2>&1
SGLM_IRLS_GROUP_MIN=4 timeout -k 10 300 python tools/rank_sim.py --world 8 --all > $O/g2.log 2>&1
SGLM_IRLS_GROUP_MIN=4 timeout -k 10 300 python tools/rank_sim.py --world 4 --all > $O/g2_w4.log 2>&1
timeout -k 10 300 python tools/rank_sim.py --world 4 --all > $O/g1_w4.log 2>&1
