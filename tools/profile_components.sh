#!/bin/bash
# Profile the standalone Ed25519 / Sum6KES / VRF kernels (bench.py
# --components-only) on the GPU box, like tools/profile.sh does the header
# kernel (run under gpurun from the repo root):
#   1. kernel trace + stats over 1M items per launch     -> gpurun_out/cprof_$TAG
#   2. FETCH_SIZE, WRITE_SIZE (HBM bytes, separate passes) -> gpurun_out/cpmc_{fetch,write}_$TAG
#   3. SQ instruction/cycle and wait counters            -> gpurun_out/cpmc_{sq,wait}_$TAG
# Every step has its own time limit; the chain stops at the first failure.
set -euo pipefail
TAG=${1:-r03}
ITEMS=${ITEMS:-262144}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --components-only --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cprof_$TAG -o run \
  -- $B --headers 1048576 --steps 3 > gpurun_out/cprof_$TAG.bench.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/cpmc_fetch_$TAG -o run \
  -- $B --headers $ITEMS --steps 1 > /dev/null
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/cpmc_write_$TAG -o run \
  -- $B --headers $ITEMS --steps 1 > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/cpmc_sq_$TAG -o run \
  -- $B --headers $ITEMS --steps 1 > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/cpmc_wait_$TAG -o run \
  -- $B --headers $ITEMS --steps 1 > /dev/null
echo profile-components-done
