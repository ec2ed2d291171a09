set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=ouroboros-network_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_claims.py tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/t2.log 2>&1
echo tests-ok
timeout -k 10 600 python tools/ab_variants.py $V/cur.so $V/bit.so --legs hdr,ed,kes,vrf --rounds 3 > gpurun_out/ab_thr2.json 2> gpurun_out/ab_thr2.err
echo abthr-ok
timeout -k 10 500 python tools/ab_latency.py --libs $V/cur.so $V/bit.so --iters 3000 --rounds 3 > gpurun_out/ab_lat2.json 2> gpurun_out/ab_lat2.err
echo ablat-ok
