set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_claims.py tests/test_gpu_concurrency.py -x -q --timeout 300 --timeout-method thread -m gpu -k "lowlat or latency or plan or counters or concurrency or golden" > gpurun_out/t3.log 2>&1
echo tests-ok
timeout -k 10 400 python tools/ab_latency.py --var OURO_PLAN_ZEROCOPY --values 0,2 --iters 3000 --rounds 3 > gpurun_out/ab_zc.json 2>&1
echo ab-ok
