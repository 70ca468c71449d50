set -u
# (run from tools/: also copy tools/labs/e2e_pinned_sweep.py to tools/ with its REPO one directory up)
# staging chunk ramp on / off, pageable and pinned host arrays, alternating in fresh processes
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/e2e_ramp_ab.txt; : > $O
for rep in 1 2 3; do for r in 1 0; do
  echo -n "ramp=$r pageable " >> $O
  SHMEMX_STAGE_RAMP=$r E2E_REPS=15 timeout -k 10 120 python3 tools/e2e_sweep.py 2>/dev/null | grep GiB >> $O || exit 1
  echo -n "ramp=$r pinned " >> $O
  SHMEMX_STAGE_RAMP=$r timeout -k 10 120 python3 tools/e2e_pinned_sweep.py 2>/dev/null | grep GiB >> $O || exit 1
done; done
cat $O
