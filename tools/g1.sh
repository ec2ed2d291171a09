set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_claims.py -x -v --timeout 300 --timeout-method thread -m gpu -k "lowlat or latency or plan or golden or counters" > gpurun_out/t1.log 2>&1
echo tests-ok
V=ouroboros-network_amd/lib/variants
timeout -k 10 400 python tools/ab_latency.py --libs $V/nosha.so $V/sha.so $V/w1.so --iters 2000 --rounds 3 > gpurun_out/ab1.json 2> gpurun_out/ab1.err
echo ab-ok
