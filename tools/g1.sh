set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_claims.py tests/test_gpu_wide.py -v --timeout 300 --timeout-method thread -m gpu -k "lowlat or latency or plan or golden or counters or wide or single_item or small or vrf" > gpurun_out/t1.log 2>&1 || echo TESTS-FAILED
echo tests-done
V=ouroboros-network_amd/lib/variants
timeout -k 10 500 python tools/ab_latency.py --libs $V/new2.so $V/new3.so $V/nosplit2.so --iters 3000 --rounds 3 > gpurun_out/ab1.json 2> gpurun_out/ab1.err
echo ab-ok
timeout -k 10 300 python tools/lat_stamps.py --runs 30 > gpurun_out/stamps4.txt 2>&1
echo stamps-ok
