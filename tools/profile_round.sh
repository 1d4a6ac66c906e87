#!/bin/bash
# Round profile on the GPU box: the default bench command under rocprofv3 kernel tracing, then two
# separate PMC passes (FETCH_SIZE, WRITE_SIZE cannot share a pass on gfx950) of a shorter bench, then
# the MFMA pass of the MPC leg.  Each pass writes the bench's launch manifest (--detail-out) beside
# its database, so tools/prof_summary.py keys every dispatch by its workload.
# Outputs under gpurun_out/; summarise with `python tools/prof_summary.py gpurun_out profiles/<round>`.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out
mkdir -p $OUT/prof_kt $OUT/prof_fetch $OUT/prof_write $OUT/prof_mfma
cd /tmp && export TMPDIR=/tmp
SHORT="--no-cpu-baseline --steps 3 --warmup 1 --rrt-steps 1 --a3-steps 2 --track-steps 1 --control-steps 2 --graph-steps 2 --dstar-steps 2 --dyn3d-steps 2"
[ "${SKIP_KT:-0}" = 1 ] || timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $OUT/prof_kt -o run -- python3 $R/bench.py \
    --detail-out $OUT/prof_kt/detail.json > $OUT/bench_prof.json 2> $OUT/bench_prof.err
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -d $OUT/prof_fetch -o run -- python3 $R/bench.py $SHORT \
    --detail-out $OUT/prof_fetch/detail.json > $OUT/bench_fetch.json 2> $OUT/bench_fetch.err
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -d $OUT/prof_write -o run -- python3 $R/bench.py $SHORT \
    --detail-out $OUT/prof_write/detail.json > $OUT/bench_write.json 2> $OUT/bench_write.err
# MFMA utilisation of the MPC tracking kernel (track_kernel<1>): its own pass
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES -d $OUT/prof_mfma -o run \
    -- python3 $R/bench.py --no-cpu-baseline --legs mpc --steps 1 --warmup 1 --track-steps 2 \
    --detail-out $OUT/prof_mfma/detail.json > $OUT/bench_mfma.json 2> $OUT/bench_mfma.err
echo profile-done
