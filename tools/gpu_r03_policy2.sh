# Round 3: the store's sc0 bit, focused (tools/policy_lab.hip list 1), warm
# and cold at 32 Mi doubles, cold at 64 Mi, twice each.
set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
{
  for i in 1 2; do
    timeout -k 10 120 tools/policy_lab 33554432 0 1
    timeout -k 10 120 tools/policy_lab 33554432 1 1
    timeout -k 10 120 tools/policy_lab 67108864 1 1
  done
} > gpurun_out/policy_lab2.txt 2>&1
cat gpurun_out/policy_lab2.txt
