#!/bin/bash
# round 5, call 11: the PMC passes of the round profile (FETCH_SIZE, WRITE_SIZE, MFMA) and an SQ issue
# pass of the A* headline kernel
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c11
ROUND=r5 PASSES=pmc timeout -k 10 1000 bash tools/profile_round.sh > gpurun_out/c11/prof.log 2>&1 || { tail -20 gpurun_out/c11/prof.log; tail -20 gpurun_out/bench_fetch.err; exit 1; }
tail -2 gpurun_out/c11/prof.log
cd /tmp && export TMPDIR=/tmp
P1=SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD
timeout -s KILL 240 rocprofv3 --pmc ${P1//,/ } -d $R/gpurun_out/c11/mq_p1 -o run -- python3 $R/bench.py --legs none --no-cpu-baseline \
  --steps 20 --warmup 5 --detail-out $R/gpurun_out/c11/mq_p1.json > $R/gpurun_out/c11/mq_p1.log 2>&1 || { echo "mq pass failed"; tail -5 $R/gpurun_out/c11/mq_p1.log; exit 1; }
python3 $R/tools/pmc_sum.py $R/gpurun_out/c11/mq_p1 mqu_kernel > $R/gpurun_out/c11/mq_issue.txt
cat $R/gpurun_out/c11/mq_issue.txt
rm -rf $R/gpurun_out/c11/mq_p1
