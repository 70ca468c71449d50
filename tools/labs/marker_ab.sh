set -u
# the host-signal marker after RCCL work: a one-thread kernel (0) or the stream's value write (1)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/marker_ab.txt; : > $O
for rep in 1 2; do for w in 0 1; do
  echo "## SHMEMX_SIGNAL_WRITEVALUE=$w rep $rep (one-rank RCCL all-reduce, SHMEMX_FORCE_COLLECTIVE=1)" >> $O
  SHMEMX_FORCE_COLLECTIVE=1 SHMEMX_SIGNAL_WRITEVALUE=$w timeout -k 10 120 python3 tools/small_call_probe.py 3000 2>/dev/null | tail -1 >> $O || exit 1
done; done
cat $O
