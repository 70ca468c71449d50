set -u
# the pageable host-resident path with the spread placement: copy threads 8 / 16 / 12 / 6
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/e2e_threads_ab.txt; : > $O
for rep in 1 2 3; do for th in 8 16 12 6; do
  SHMEMX_COPY_THREADS=$th E2E_REPS=15 timeout -k 10 120 python3 tools/e2e_sweep.py 2>/dev/null | grep GiB >> $O || exit 1
done; done
echo "cpu.stat: $(grep -E 'nr_throttled|throttled_usec' /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' ')" >> $O
cat $O
