# Round-6: structured Gram -- MFMA bursts at raised wave priority (SGLM_LAGW_PRIO=1) against the
# default; parity tests after the Hb tile staging in the symmetrize pass.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-prio}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_laggram_w.py > $O/tests.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_base.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LAGW_PRIO=1 python3 tools/lagw_bench.py > $O/time_prio.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_base2.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LAGW_PRIO=1 python3 tools/lagw_bench.py > $O/time_prio2.log 2>&1
echo done
