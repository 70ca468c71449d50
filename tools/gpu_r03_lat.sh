# Round 3: small-call latency A/B, host signals on and off (SHMEMX_HOST_SIGNAL).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for hs in 1 0 1 0; do
  echo "SHMEMX_HOST_SIGNAL=$hs"
  SHMEMX_HOST_SIGNAL=$hs bash tools/gpu_latency_cmp.sh || exit $?
done
SHMEMX_HOST_SIGNAL=1 timeout -k 10 120 ./tools/latency_breakdown | grep api
SHMEMX_HOST_SIGNAL=0 timeout -k 10 120 ./tools/latency_breakdown | grep api
