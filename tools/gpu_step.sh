# one GPU call: tracking tests (four agents per wave), then the lqr/mpc legs at 2048 and 8192 agents
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_track_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_trk1.log 2>&1 && \
timeout -k 10 300 python bench.py --legs lqr,mpc --no-cpu-baseline --steps 1 --warmup 1 --detail-out gpurun_out/r3_trk1_2048.json > /dev/null 2> gpurun_out/r3_trk1.err && \
timeout -k 10 300 python bench.py --legs lqr,mpc --no-cpu-baseline --steps 1 --warmup 1 --track-agents 8192 --detail-out gpurun_out/r3_trk1_8192.json > /dev/null 2>> gpurun_out/r3_trk1.err
