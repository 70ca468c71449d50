set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/kernarg_ab.txt; : > $O
for rep in 1 2; do for k in unset 0 1; do
  if [ $k = unset ]; then envs=""; else envs="HIP_FORCE_DEV_KERNARG=$k"; fi
  echo "## HIP_FORCE_DEV_KERNARG=$k rep $rep" >> $O
  env $envs timeout -k 10 120 python3 tools/small_call_probe.py 3000 >> $O 2>>gpurun_out/kernarg.err || exit 1
done; done
cat $O
