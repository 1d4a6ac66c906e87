#!/bin/bash
# round 6, call 50: RRT* phase stamps at 256 threads x 2 per CU (512 queries: every CU busy)
# result (phase shares at 512 queries, 2 per CU): nearest loop 9 %, reduce 6 %, band 1 %, steer + collision 30 %, radius stage 5 %, resolve 7 %, tests + choose + rewire 38 %, insert + goal 5 %
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R
PMP_HIP_LIB=$L/libpmp_hip_rrtstamps2.so timeout -k 10 300 python3 -u tools/rrt_time.py 512x65536 2>&1 | grep -A3 "phase shares\|nq=" || exit 1
