# Grid A/B of the per-launch kernel switches for the gradient and direction products
# (tools/grid_ab.py, one process, alternating grids).  Usage on the box: bash tools/gpu_knobs_ab.sh
set -e
export TMPDIR=/tmp
O=gpurun_out/knobs; mkdir -p $O
timeout -k 10 600 python -u tools/grid_ab.py 6 base: etadir1:env.SGLM_ETA_DIR=1 etadir0:env.SGLM_ETA_DIR=0 xtr3:env.SGLM_XTR_NGW=3 nococh:XTR_COCHAIN=False nolag:LAG_GRAM=False > $O/ab.json 2> $O/ab.err
