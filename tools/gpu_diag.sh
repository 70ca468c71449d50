set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
grep -E "^(Name|Marketing)" <(rocminfo 2>/dev/null) | head -4
timeout -k 10 120 python tools/diag_init.py no_torch > gpurun_out/diag_notorch.log 2>&1; echo "no_torch rc=$?"; tail -5 gpurun_out/diag_notorch.log
AMD_LOG_LEVEL=3 timeout -k 10 180 python tools/diag_init.py torch_first > gpurun_out/diag_torch.log 2>&1; echo "torch_first rc=$?"; grep -v "^:3:" gpurun_out/diag_torch.log | tail -8; grep -E ":1:|:2:|rror|fail" gpurun_out/diag_torch.log | tail -20
