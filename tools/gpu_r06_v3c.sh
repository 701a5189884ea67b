# Round-6: structured Gram v3 with the register file held whole (256 VGPRs) against v3 at ~220
# VGPRs and the previous kernel: C4 grids interleaved, standalone timing, kernel trace.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-v3c}; mkdir -p $O
V=sabatinilab-glm_amd/sglm_hip/variants
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_new.log 2>&1
for k in 1 2; do
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_new$k.json 2> $O/bench_new$k.err
timeout -k 10 300 env SGLM_LIB=$V/libsglm_v3b.so python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_v3b$k.json 2> $O/bench_v3b$k.err
timeout -k 10 300 env SGLM_LIB=$V/libsglm_prev.so python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_prev$k.json 2> $O/bench_prev$k.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-dropin --no-check > $O/bench_prof.json 2> $O/kt.err
echo done
