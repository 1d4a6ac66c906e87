# one GPU call: the GPU test suite, then the default bench
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gputest6.log 2>&1 && \
timeout -k 10 700 python bench.py --detail-out gpurun_out/r3_bench6_detail.json > gpurun_out/r3_bench6.json 2> gpurun_out/r3_bench6.err
