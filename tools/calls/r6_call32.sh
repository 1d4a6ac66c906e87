#!/bin/bash
# round 6, call 32: RRT* coarse scans on exact 15-bit integer distances (pk_sub_i16 + dot2; vs the f32 decode form) + tests the segment while the other waves stage the
# in-radius hits around the nearest node) -- RRT parity, A/B against the committed kernel, stamps, bench leg
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c32
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_rrt_gpu.py \
  > gpurun_out/r6c32/pytest.log 2>&1 || { tail -30 gpurun_out/r6c32/pytest.log; exit 1; }
tail -1 gpurun_out/r6c32/pytest.log
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export PMP_HIP_LIB=$L/libpmp_hip_rrtold.so; else unset PMP_HIP_LIB; fi
    echo "== $v round $r: $(timeout -k 10 200 python3 -u tools/rrt_time.py 256x65536 2>&1 | grep 'nq=')"
  done
done
unset PMP_HIP_LIB

timeout -k 10 300 python3 bench.py --legs rrt --steps 2 --warmup 1 --no-cpu-baseline --detail-out gpurun_out/r6c32/d.json \
  > gpurun_out/r6c32/b.out 2> gpurun_out/r6c32/b.err || { tail -20 gpurun_out/r6c32/b.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r6c32/b.out').read().strip().splitlines()[-1]); print('bench rrt_star', d['secondary']['rrt_star']['value'])"
PMP_HIP_LIB=$L/libpmp_hip_rrtstamps2.so timeout -k 10 300 python3 -u tools/rrt_time.py 256x65536 2>&1 | grep "phase shares" || exit 1
