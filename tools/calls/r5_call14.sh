#!/bin/bash
# round 5, call 14: launch-time variation -- repeated launches on one context vs fresh contexts
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c14
timeout -k 10 400 python3 tools/launch_repeat.py theta_star 12 32 3 3 > gpurun_out/c14/theta.log 2>&1 || { tail -20 gpurun_out/c14/theta.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c14/theta.log
timeout -k 10 400 python3 tools/launch_repeat.py astar 20 60 2 3 > gpurun_out/c14/astar.log 2>&1 || { tail -20 gpurun_out/c14/astar.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c14/astar.log
