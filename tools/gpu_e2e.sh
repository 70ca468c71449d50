set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for th in 4 8 16 32; do for ch in 4 8 16 32; do
  SHMEMX_COPY_THREADS=$th SHMEMX_STAGE_CHUNK_MB=$ch timeout -k 10 120 python tools/e2e_sweep.py || exit 1
done; done
