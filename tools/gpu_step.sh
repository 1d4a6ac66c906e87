# one GPU call (edit per experiment); long outputs under gpurun_out/
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_astar2d_gpu.py -x -v --timeout 300 --timeout-method thread -k "residency or dropin" > gpurun_out/r3_gputest3.log 2>&1 && \
timeout -k 10 300 python bench.py --legs none --detail-out gpurun_out/r3_b_mq.json > gpurun_out/r3_bench_mq.json 2> gpurun_out/r3_bench_mq.err && \
timeout -k 10 300 python bench.py --legs none --t2lds 1 --residency 32 --detail-out gpurun_out/r3_b_mqt2.json > gpurun_out/r3_bench_mqt2.json 2> gpurun_out/r3_bench_mqt2.err
