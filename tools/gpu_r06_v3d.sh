# Round-6: in-process interleaved A/B of the structured Gram holding 256 VGPRs (default) against
# ~220 (SGLM_LAGW_HOLD=0), C4 grid; standalone timings both ways.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-v3d}; mkdir -p $O
timeout -k 10 600 python3 tools/grid_ab.py 8 hold:env.SGLM_LAGW_HOLD=1 free:env.SGLM_LAGW_HOLD=0 > $O/ab_hold.json 2> $O/ab_hold.err
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_hold.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LAGW_HOLD=0 python3 tools/lagw_bench.py > $O/time_free.log 2>&1
echo done
