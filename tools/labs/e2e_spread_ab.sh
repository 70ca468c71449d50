set -u
# the pageable host-resident path: copy gangs placed by the scheduler (all) or
# one per cache domain of the GPU's node (spread), alternating in fresh processes
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/e2e_spread_ab.txt; : > $O
echo "loadavg: $(cat /proc/loadavg)" >> $O
SHMEMX_COPY_CPUS=spread SHMEM_LOG_LEVELS=INFO E2E_REPS=3 timeout -k 10 120 python3 tools/e2e_sweep.py 2>&1 | grep -E "cache domain|GiB/s" >> $O || exit 1
for rep in 1 2 3 4; do for m in all spread; do
  echo -n "cpus=$m " >> $O
  SHMEMX_COPY_CPUS=$m E2E_REPS=15 timeout -k 10 120 python3 tools/e2e_sweep.py 2>/dev/null | grep GiB >> $O || exit 1
done; done
echo "loadavg: $(cat /proc/loadavg)" >> $O
cat $O
