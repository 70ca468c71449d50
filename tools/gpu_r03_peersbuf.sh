# Round 3: the P = 8 fold with buffer loads (tools/peers_buf_lab.hip), at
# 16 Mi and 4 Mi doubles per input.
set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
{
  timeout -k 10 120 tools/peers_buf_lab 16777216
  timeout -k 10 120 tools/peers_buf_lab 4194304
} > gpurun_out/peers_buf_lab.txt 2>&1
cat gpurun_out/peers_buf_lab.txt
