#!/bin/bash
# PMC issue/latency breakdown of the A* 2D kernel on the C2 batch (tools/astar2d_one.py MODE=batch).
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=${OUT:-$R/gpurun_out/pmc_issue}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
S1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM"
S2="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
S3="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_CYCLES"
i=0
for set in "$S1" "$S2" "$S3"; do
  i=$((i+1))
  MODE=batch timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/batch_$i -o run -- python3 $R/tools/astar2d_one.py > $OUT/batch_$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo pmc-done
