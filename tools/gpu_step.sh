# one GPU call: register-inverse build under the tracking tests + mpc leg, then the LDS default's mpc leg
cd $GRAFT_REPO_ROOT
export PMPR=$GRAFT_REPO_ROOT/python_motion_planning_amd/libpmp_hip_invreg.so
PMP_HIP_LIB=$PMPR timeout -k 10 300 python -u -m pytest tests/test_track_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_t12.log 2>&1 && \
PMP_HIP_LIB=$PMPR timeout -k 10 300 python bench.py --legs mpc --no-cpu-baseline --steps 2 --warmup 1 --detail-out gpurun_out/r3_b12r.json > /dev/null 2> gpurun_out/r3_b12.err && \
timeout -k 10 300 python bench.py --legs mpc --no-cpu-baseline --steps 2 --warmup 1 --detail-out gpurun_out/r3_b12l.json > /dev/null 2>> gpurun_out/r3_b12.err && \
PMP_HIP_LIB=$PMPR timeout -k 10 300 python bench.py --legs mpc --no-cpu-baseline --steps 2 --warmup 1 --track-agents 32768 --detail-out gpurun_out/r3_b12r32.json > /dev/null 2>> gpurun_out/r3_b12.err
