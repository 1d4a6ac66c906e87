#!/bin/bash
# round 6, call 20: RRT* C3 per-query iteration distribution (is the launch held by a few queries?)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/r6c20
timeout -k 10 300 python3 -u tools/rrt_time.py 256x65536 2>&1 | grep -v amdgpu.ids || exit 1
