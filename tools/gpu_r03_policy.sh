# Round 3: cache-policy bits of the 2-input fold (tools/policy_lab.hip), warm
# and cold, at the bench size (32 Mi doubles) and at 64 Mi.
set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
{
  timeout -k 10 120 tools/policy_lab 33554432 0
  timeout -k 10 120 tools/policy_lab 33554432 1
  timeout -k 10 120 tools/policy_lab 67108864 0
} > gpurun_out/policy_lab.txt 2>&1
cat gpurun_out/policy_lab.txt
