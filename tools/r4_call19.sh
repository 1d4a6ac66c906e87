#!/bin/bash
# round 4, call 19: 3D A* residency below 20 per CU, and a build for 4 waves per SIMD at 16 per CU
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c19
run() {  # tag lib residency
  PMP_HIP_LIB=$R/python_motion_planning_amd/$2 timeout -k 10 200 python3 bench.py --legs astar3d --no-cpu-baseline --steps 1 --warmup 1 --a3-residency $3 > gpurun_out/c19/$1.json 2> gpurun_out/c19/$1.err || { tail -5 gpurun_out/c19/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c19/$1.json').read().strip().splitlines()[-1]); print('$1', d['secondary']['astar3d']['value'])"
}
for i in 1 2; do
  run r20_$i libpmp_hip.so 20
  run r16_$i libpmp_hip.so 16
  run r18_$i libpmp_hip.so 18
  run w4r16_$i libpmp_hip_a3w4.so 16
done
