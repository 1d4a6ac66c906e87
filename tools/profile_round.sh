#!/bin/bash
# Round profile on the GPU box: the default bench command under rocprofv3 kernel tracing, then two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE cannot share a pass on gfx950) of a shorter bench, then
# the MFMA pass of the MPC leg.  Each pass writes the bench's launch manifest (--detail-out) beside
# its database, so tools/prof_summary.py keys every dispatch by its workload.
# The PMC passes keep the default per-launch batch counts of the multi-batch legs (the A* headline's
# 20 batches in one launch, 3D A*'s 32), so a dispatch there is the same work as in the default run;
# (Theta* 12 and DStar3D / LPAStar3D 6 batches per launch too); the other legs are shortened (fewer
# launches of the same size).
# Outputs under gpurun_out/; the summary is written on the box (ROUND=r3 -> gpurun_out/profiles_r3)
# and the databases are deleted (they would exceed gpurun_out's 64 MiB).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT/prof_kt $OUT/prof_fetch $OUT/prof_write $OUT/prof_mfma $OUT/prof_issue
cd /tmp && export TMPDIR=/tmp
SHORT="--no-cpu-baseline --warmup 1 --rrt-steps 1 --track-steps 1 --control-steps 2 --graph-steps 12 --dstar-steps 2 --dyn3d-steps 6"
# PASSES=kt / pmc / issue / all (separate gpurun calls fit the per-call limit better than one)
P=${PASSES:-all}
[ "$P" = pmc ] || [ "$P" = issue ] || timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $OUT/prof_kt -o run -- python3 $R/bench.py --steps 20 --warmup 5 \
    --detail-out $OUT/prof_kt/detail.json > $OUT/bench_prof.json 2> $OUT/bench_prof.err
if [ "$P" = pmc ] || [ "$P" = all ]; then
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run -- python3 $R/bench.py $SHORT \
    --detail-out $OUT/prof_fetch/detail.json > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run -- python3 $R/bench.py $SHORT \
    --detail-out $OUT/prof_write/detail.json > $OUT/bench_write.json 2> $OUT/bench_write.err
fi
if [ "$P" = issue ] || [ "$P" = all ]; then
# the SQ issue pass (8 SQ + 1 GRBM counters: within one pass's limits)
timeout -k 10 500 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/prof_issue -o run -- python3 $R/bench.py $SHORT \
    --detail-out $OUT/prof_issue/detail.json > $OUT/bench_issue.json 2> $OUT/bench_issue.err
# MFMA utilisation of the MPC tracking kernels (track_mpc_solve carries the assembly): its own pass
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $OUT/prof_mfma -o run \
    -- python3 $R/bench.py --no-cpu-baseline --legs mpc --steps 1 --warmup 1 --track-steps 2 \
    --detail-out $OUT/prof_mfma/detail.json > $OUT/bench_mfma.json 2> $OUT/bench_mfma.err
fi
python3 $R/tools/prof_summary.py $OUT $OUT/profiles_${ROUND:-r3} > $OUT/prof_summary.log 2>&1
rm -rf $OUT/prof_kt/*/ $OUT/prof_fetch/*/ $OUT/prof_write/*/ $OUT/prof_mfma/*/ $OUT/prof_issue/*/ $OUT/prof_kt/*.db \
    $OUT/prof_fetch/*.db $OUT/prof_write/*.db $OUT/prof_mfma/*.db $OUT/prof_issue/*.db
echo profile-done
