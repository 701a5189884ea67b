# Round-6b: device-side Newton decisions (sglm_step_decide, the step and the next link enqueued
# before the readback) against the host decisions, at the 29 ms grid
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-devdec}; mkdir -p $O
timeout -k 10 600 python3 -u tools/grid_ab.py 8 base: dev:DEV_DECIDE=True > $O/ab.json 2> $O/ab.err
echo done
