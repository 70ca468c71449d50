# long randomized multi-PE soak on both transports (tests/gpu_ipc_child.py "soak")
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for seed in 11 12 13; do
  SOAK_ITERS=1500 SOAK_SEED=$seed timeout -k 10 600 python -u -m pytest tests/test_gpu_ipc.py -k soak -x -q \
    --timeout 580 --timeout-method thread --basetemp=gpurun_out/soak_$seed > gpurun_out/soak_$seed.log 2>&1
  rc=$?; echo "seed $seed rc=$rc: $(tail -1 gpurun_out/soak_$seed.log)"
  [ $rc -eq 0 ] || exit $rc
done
for d in gpurun_out/soak_11/*/; do echo "$d: $(python3 -c "import json,glob; print([json.load(open(f))['ncases'] for f in sorted(glob.glob('$d/pe*.json'))])")"; done
