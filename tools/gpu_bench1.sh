set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench1.log 2>&1; rc=$?
grep '"metric"' gpurun_out/bench1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['extras'], indent=1))"
exit $rc
