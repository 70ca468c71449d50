# Round 3: fold_peers_kernel with buffer loads (SHMEMX_PEERS_BUFFER=1) against
# global loads (=0): the peers-fold tests under the buffer path, then the
# local-HBM rate of both, twice, interleaved.
set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SHMEMX_PEERS_BUFFER=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_golden.py -m gpu -x -q --timeout 240 --timeout-method thread -k "peers or fuzz or reference" > gpurun_out/peersbuf_tests.log 2>&1
tail -3 gpurun_out/peersbuf_tests.log
for i in 1 2; do
  for b in 0 1; do
    echo "== SHMEMX_PEERS_BUFFER=$b (pass $i)"
    SHMEMX_PEERS_BUFFER=$b timeout -k 10 180 python -u tools/fold_n_probe.py
  done
done > gpurun_out/peersbuf_ab.txt 2>&1
cat gpurun_out/peersbuf_ab.txt
