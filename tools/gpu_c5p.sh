set -e
O=gpurun_out/c5; mkdir -p $O
timeout -k 10 400 python tools/c5_probe.py --responses 64 --alphas 20 > $O/probe1.txt 2>&1
timeout -k 10 400 python -c "
import cProfile, pstats, sys, runpy
sys.argv=['c5_probe.py','--responses','64','--alphas','20']
sys.path[:0]=['tools']
import c5_probe
c5_probe.main()
pr=cProfile.Profile(); pr.enable(); c5_probe.main(); pr.disable()
st=pstats.Stats(pr); st.sort_stats('cumtime').print_stats(35)
" > $O/cprof2.txt 2>&1
