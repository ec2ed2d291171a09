set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=ouroboros-network_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/t6.log 2>&1
echo tests-ok
timeout -k 10 500 python tools/ab_variants.py $V/nopack.so $V/pack.so --rounds 3 --legs hdr,ed,kes,vrf > gpurun_out/ab_pack.json 2>&1
echo ab-ok
timeout -k 10 500 bash tools/pmc_variants.sh pack $V/nopack.so $V/pack.so > gpurun_out/pmc_pack.log 2>&1
echo pmc-ok
