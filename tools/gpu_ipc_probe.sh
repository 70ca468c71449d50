set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for np in 2 4; do
  f=/dev/shm/ipcprobe.$$.$np; pids=()
  for ((p=0;p<np;p++)); do timeout -k 5 90 tools/ipc_probe $p $np $f & pids+=($!); done
  rc=0; for pid in "${pids[@]}"; do wait $pid || rc=$?; done
  echo "np=$np rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
