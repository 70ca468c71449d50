# Round 2: the P-input fold lab over input layouts (one block at k*(n*8+skew)),
# then counters for every shipped kernel (tools/gpu_pmc_all.sh).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for a in "4194304 0 0" "4194304 0 4096" "4194304 0 65792" "4194304 0 2101248" "4194304 1 0" "4194304 1 65792"; do
  timeout -k 10 120 ./tools/foldn_lab $a >> gpurun_out/foldn_skew.txt 2>&1 || { echo "lab failed $?"; tail -5 gpurun_out/foldn_skew.txt; exit 1; }
done
grep -E "^#|rt_u4|pipe_u4|st_u4|rdonly" gpurun_out/foldn_skew.txt
bash tools/gpu_pmc_all.sh r02
