# pinned host-resident end-to-end rate vs staging chunk size, plus raw PCIe rates
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
RAW=1 timeout -k 10 120 python tools/e2e_pinned_sweep.py > gpurun_out/e2e_pinned.txt 2>&1 || exit 1
for mb in 2 4 8 32 64; do
  SHMEMX_STAGE_CHUNK_MB=$mb timeout -k 10 120 python tools/e2e_pinned_sweep.py >> gpurun_out/e2e_pinned.txt 2>&1 || exit 1
done
cat gpurun_out/e2e_pinned.txt | grep chunkMB
