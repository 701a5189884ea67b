# Run GPU steps in order, each under its own time limit; stop at the first step that faulted,
# aborted, crashed or timed out (rc 124/134/137/139 or > 128), continue past plain test
# failures (rc 1).  Usage: bash tools/gpu_step.sh OUTDIR 'cmd1' 'cmd2' ...  (each cmd is run as
# "timeout -k 10 <secs> <cmd>" where the first word of cmd is the seconds)
export TMPDIR=/tmp
O=$1; shift
mkdir -p $O
i=0
for c in "$@"; do
  i=$((i+1))
  secs=${c%% *}; cmd=${c#* }
  echo "== step $i: $cmd" | tee -a $O/steps.log
  timeout -k 10 $secs bash -c "$cmd" > $O/step$i.out 2> $O/step$i.err
  rc=$?
  echo "rc=$rc" | tee -a $O/steps.log
  tail -3 $O/step$i.out | tee -a $O/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc" | tee -a $O/steps.log; exit $rc; fi
done
