#!/bin/bash
# PMC issue/latency breakdown of an A* 2D engine on the C2 batch (tools/astar2d_probe.py, REPS=1):
# three separate rocprofv3 --pmc passes; summary by tools/pmc_probe_read.py.  TAG names the output.
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=${OUT:-$R/gpurun_out/pmc_${TAG:-probe}}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
S1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS"
S2="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"
S3="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_CYCLES"
i=0
for set in "$S1" "$S2" "$S3"; do
  i=$((i+1))
  REPS=1 timeout -s KILL 150 rocprofv3 --pmc $set -d $OUT/p$i -o run -- python3 $R/tools/astar2d_probe.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
python3 $R/tools/pmc_probe_read.py $OUT > $OUT/summary.txt && rm -rf $OUT/p1 $OUT/p2 $OUT/p3
echo pmc-done
