set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=ouroboros-network_amd/lib/variants
timeout -k 10 500 python tools/ab_variants.py $V/pack.so $V/pf0.so --rounds 3 --legs hdr,ed,kes,vrf > gpurun_out/ab_pf0.json 2>&1
echo ab-ok
timeout -k 10 300 bash tools/pmc_variants.sh pf0 $V/pf0.so > gpurun_out/pmc_pf0.log 2>&1
echo pmc-ok
