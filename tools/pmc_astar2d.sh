#!/bin/bash
# PMC instruction mix of the A* 2D kernel (tools/astar2d_one.py), one pass per counter set.
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc_a2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
S1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
S2="SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU_FP64"
for mode in ${MODES:-longest batch}; do
  i=0
  for set in "$S1" "$S2"; do
    i=$((i+1))
    MODE=$mode timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/${mode}_$i -o run -- python3 $R/tools/astar2d_one.py > $OUT/${mode}_$i.log 2>&1 || { echo "pass $mode $i failed rc=$?"; exit 1; }
  done
done
echo pmc-done
