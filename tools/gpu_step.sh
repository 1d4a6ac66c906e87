# one GPU call: tracking tests with the split MPC (step / solve kernels), then the mpc leg at 8192 / 32768 agents
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_track_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3_t13.log 2>&1 && \
timeout -k 10 300 python bench.py --legs mpc --no-cpu-baseline --steps 2 --warmup 1 --track-agents 8192 --detail-out gpurun_out/r3_b13a.json > /dev/null 2> gpurun_out/r3_b13.err && \
timeout -k 10 300 python bench.py --legs mpc --no-cpu-baseline --steps 2 --warmup 1 --detail-out gpurun_out/r3_b13b.json > /dev/null 2>> gpurun_out/r3_b13.err
