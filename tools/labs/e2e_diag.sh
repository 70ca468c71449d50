set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/e2e_diag.txt
{
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "loadavg: $(cat /proc/loadavg)"; nproc
echo "cpu.stat before:"; cat /sys/fs/cgroup/cpu.stat 2>/dev/null | head -6
} > $O 2>&1
for th in 8 4 16 8; do
  SHMEMX_COPY_THREADS=$th E2E_REPS=11 timeout -k 10 120 python3 tools/e2e_sweep.py >> $O 2>&1 || exit 1
  echo "cpu.stat: $(grep -E 'nr_throttled|throttled_usec' /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' ')" >> $O
done
echo "loadavg: $(cat /proc/loadavg)" >> $O
cat $O
