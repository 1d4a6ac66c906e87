#!/bin/bash
# round 6, call 47: D* heap / entry capacity per cell 4 (the bound) vs 2 vs 1: overflow counts and one
# launch's time at 256^2 / 512^2 (4096 queries, one context)
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R
for v in def hpc2 hpc1; do
  if [ $v = def ]; then unset PMP_HIP_LIB; else export PMP_HIP_LIB=$L/libpmp_hip_$v.so; fi
  echo "== $v"; timeout -k 10 300 python3 -u tools/dstar_cap_probe.py || exit 1
done
