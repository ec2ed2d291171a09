set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=ouroboros-network_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/t8.log 2>&1
echo tests-ok
timeout -k 10 500 python tools/ab_variants.py $V/noid0.so $V/id0.so --rounds 3 --legs hdr,ed,kes,vrf > gpurun_out/ab_id0.json 2>&1
echo ab-ok
