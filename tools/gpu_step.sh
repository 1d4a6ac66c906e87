# one GPU call: tracking + 3D + D* tests, then lqr/mpc/astar3d legs (multi-batch 3D launches) and A/B variants
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_track_gpu.py tests/test_astar3d_gpu.py tests/test_dstar_gpu.py tests/test_dstar3d_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_t9.log 2>&1 && \
timeout -k 10 300 python bench.py --legs lqr,mpc,astar3d --no-cpu-baseline --steps 1 --warmup 1 --detail-out gpurun_out/r3_b9a.json > /dev/null 2> gpurun_out/r3_b9.err && \
PMP_HIP_LIB=$GRAFT_REPO_ROOT/python_motion_planning_amd/libpmp_hip_invreg.so timeout -k 10 300 python bench.py --legs lqr,mpc --no-cpu-baseline --steps 1 --warmup 1 --detail-out gpurun_out/r3_b9r.json > /dev/null 2>> gpurun_out/r3_b9.err && \
timeout -k 10 300 python bench.py --legs lqr,mpc,astar3d --no-cpu-baseline --steps 1 --warmup 1 --track-agents 32768 --a3-batches-per-launch 8 --detail-out gpurun_out/r3_b9b.json > /dev/null 2>> gpurun_out/r3_b9.err && \
timeout -k 10 300 python bench.py --legs astar3d --no-cpu-baseline --steps 1 --warmup 1 --a3-residency 48 --detail-out gpurun_out/r3_b9c.json > /dev/null 2>> gpurun_out/r3_b9.err
