#!/bin/bash
# round 6, call 22: RRT* phase stamps at C3 (256 x 65,536) on the round's kernel; LPAStar3D / DStar3D
# launch schedule after the extractPath fix (batches per launch x launches in flight)
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c22
PMP_HIP_LIB=$L/libpmp_hip_rrtstamps.so timeout -k 10 300 python3 -u tools/rrt_time.py 256x65536 2>&1 | grep -v amdgpu.ids || exit 1
for cfg in "6 4" "24 1" "12 2"; do
  set -- $cfg
  timeout -k 10 400 python3 bench.py --legs dyn3d --steps 2 --warmup 1 --no-cpu-baseline --dyn3d-batches-per-launch $1 \
    --dyn3d-streams $2 --detail-out gpurun_out/r6c22/d_$1_$2.json > gpurun_out/r6c22/b_$1_$2.out 2> gpurun_out/r6c22/b_$1_$2.err \
    || { tail -20 gpurun_out/r6c22/b_$1_$2.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r6c22/b_$1_$2.out').read().strip().splitlines()[-1])
print('dyn3d batches/launch $1 streams $2:', {k: v['value'] for k, v in d['secondary'].items()})
"
done
