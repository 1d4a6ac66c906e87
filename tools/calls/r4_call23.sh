#!/bin/bash
# round 4, call 23: heap16.push_batch for D* and DStar3D (3D A* refactored onto it) -- parity of every
# heap16 user, then same-box A/B of the D* / DStar3D / 3D A* legs against the previous head
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c23
timeout -k 10 600 python -u -m pytest tests/test_astar3d_gpu.py tests/test_graph_variants_gpu.py tests/test_dstar_gpu.py tests/test_dstar3d_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c23/tests.log 2>&1 || { tail -40 gpurun_out/c23/tests.log; exit 1; }
tail -2 gpurun_out/c23/tests.log
run() {  # tag lib legs
  PMP_HIP_LIB=$R/python_motion_planning_amd/$2 timeout -k 10 300 python3 bench.py --legs $3 --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/c23/$1.json 2> gpurun_out/c23/$1.err || { tail -5 gpurun_out/c23/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c23/$1.json').read().strip().splitlines()[-1]); s=d['secondary']; print('$1', {k: s[k]['value'] for k in s})"
}
for i in 1 2; do
  run pre_$i libpmp_hip_prebd.so astar3d,dstar,dyn3d
  run new_$i libpmp_hip.so astar3d,dstar,dyn3d
done
