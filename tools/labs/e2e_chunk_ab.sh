set -u
# the pageable host-resident path (default copy placement): staging chunk size
# 16 / 8 / 4 / 32 MiB, alternating in fresh processes
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/e2e_chunk_ab.txt; : > $O
for rep in 1 2 3; do for ch in 16 8 4 32; do
  SHMEMX_STAGE_CHUNK_MB=$ch E2E_REPS=15 timeout -k 10 120 python3 tools/e2e_sweep.py 2>/dev/null | grep GiB >> $O || exit 1
done; done
cat $O
