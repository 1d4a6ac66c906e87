#!/bin/bash
# round 4, call 20: 3D A* batch store of an expansion's live neighbours (sift-up only below the parent)
# against the pre-change build and the build without it, same box, after the heap16 users' parity tests
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c20
timeout -k 10 600 python -u -m pytest tests/test_astar3d_gpu.py tests/test_graph_variants_gpu.py tests/test_dstar_gpu.py tests/test_dstar3d_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c20/tests.log 2>&1 || { tail -40 gpurun_out/c20/tests.log; exit 1; }
tail -2 gpurun_out/c20/tests.log
run() {  # tag lib residency
  PMP_HIP_LIB=$R/python_motion_planning_amd/$2 timeout -k 10 200 python3 bench.py --legs astar3d --no-cpu-baseline --steps 1 --warmup 1 --a3-residency $3 > gpurun_out/c20/$1.json 2> gpurun_out/c20/$1.err || { tail -5 gpurun_out/c20/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c20/$1.json').read().strip().splitlines()[-1]); print('$1', d['secondary']['astar3d']['value'], 'headline', round(d['value']))"
}
for i in 1 2; do
  run old_r20_$i libpmp_hip_old3d.so 20
  run nobatch_r20_$i libpmp_hip_nobatch.so 20
  run batch_r20_$i libpmp_hip.so 20
  run batch_r24_$i libpmp_hip.so 24
done
