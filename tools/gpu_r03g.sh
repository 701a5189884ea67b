# Full GPU suite, then the A/B benches of the four-panel gradient and the 128-tile inversion.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03g}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=15 -p no:cacheprovider tests -m gpu > $O/tests.log 2>&1
SGLM_XTR4=1 timeout -k 10 200 python -u tools/lag_bench.py 120,16,6 bits > $O/micro4.log 2>&1
SGLM_XTR4=0 timeout -k 10 200 python -u tools/lag_bench.py 120,16,6 bits > $O/micro1.log 2>&1
for v in base x4 i128 x4i128; do
  case $v in
    base) export SGLM_XTR4=0 SGLM_INV128_MIN=0;;
    x4) export SGLM_XTR4=1 SGLM_INV128_MIN=0;;
    i128) export SGLM_XTR4=0 SGLM_INV128_MIN=4;;
    x4i128) export SGLM_XTR4=1 SGLM_INV128_MIN=4;;
  esac
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_$v.json 2> $O/bench_$v.err
done
