#!/bin/bash
# round 6, call 29: RRT* finer phase stamps (PMP_RRT_STAMPS=2) at C3 on the round's kernel
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c29
PMP_HIP_LIB=$L/libpmp_hip_rrtstamps2.so timeout -k 10 300 python3 -u tools/rrt_time.py 256x65536 2>&1 | grep -v amdgpu.ids || exit 1
