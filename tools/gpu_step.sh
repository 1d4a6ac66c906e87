# one GPU call: dyn3d legs, one batch per launch on 6 streams vs all 24 batches in one launch / 6 per launch
cd $GRAFT_REPO_ROOT
B="python bench.py --no-cpu-baseline --steps 1 --warmup 1 --legs dyn3d"
timeout -k 10 400 $B --detail-out gpurun_out/r3_b16a.json > /dev/null 2> gpurun_out/r3_b16.err && \
timeout -k 10 400 $B --dyn3d-batches-per-launch 0 --detail-out gpurun_out/r3_b16b.json > /dev/null 2>> gpurun_out/r3_b16.err && \
timeout -k 10 400 $B --dyn3d-batches-per-launch 6 --dyn3d-streams 4 --detail-out gpurun_out/r3_b16c.json > /dev/null 2>> gpurun_out/r3_b16.err
