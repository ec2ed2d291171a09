set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=ouroboros-network_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_claims.py tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/t5.log 2>&1
echo tests-ok
timeout -k 10 400 python tools/ab_latency.py --libs $V/noell2.so $V/ell2.so --iters 3000 --rounds 4 > gpurun_out/ab_ell2.json 2>&1
echo ab-ok
