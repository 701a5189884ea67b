# A/B of the stopping rule: full-size C4 parity tests and the C4 bench grid under each rule.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-stop}; mkdir -p $O
for v in split legacy; do
  case $v in legacy) export SGLM_STOP_RULE=legacy;; split) export SGLM_STOP_RULE=;; esac
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_fullsize.py -k "c4_grid or newton" -s > $O/tests_$v.log 2>&1 || true
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_$v.json 2> $O/bench_$v.err
done
