#!/bin/bash
# round 6, call 33: RRT* DPP wave reductions (nearest top-2, choose-parent min) vs LDS-pipe permutes + tests the segment while the other waves stage the
# in-radius hits around the nearest node) -- RRT parity, A/B against the committed kernel, stamps, bench leg
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c33
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_rrt_gpu.py \
  > gpurun_out/r6c33/pytest.log 2>&1 || { tail -30 gpurun_out/r6c33/pytest.log; exit 1; }
tail -1 gpurun_out/r6c33/pytest.log
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export PMP_HIP_LIB=$L/libpmp_hip_rrtold.so; else unset PMP_HIP_LIB; fi
    echo "== $v round $r: $(timeout -k 10 200 python3 -u tools/rrt_time.py 256x65536 2>&1 | grep 'nq=')"
  done
done
unset PMP_HIP_LIB

timeout -k 10 300 python3 bench.py --legs rrt --steps 2 --warmup 1 --no-cpu-baseline --detail-out gpurun_out/r6c33/d.json \
  > gpurun_out/r6c33/b.out 2> gpurun_out/r6c33/b.err || { tail -20 gpurun_out/r6c33/b.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r6c33/b.out').read().strip().splitlines()[-1]); print('bench rrt_star', d['secondary']['rrt_star']['value'])"
PMP_HIP_LIB=$L/libpmp_hip_rrtstamps2.so timeout -k 10 300 python3 -u tools/rrt_time.py 256x65536 2>&1 | grep "phase shares" || exit 1
