#!/bin/bash
# round 6, call 15: LPAStar3D phase stamps -- the round-5 form vs deferred removes (shares and ticks
# per expansion), and the updates split into removes / pushes / compaction
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c15
for v in stamps_old stamps stamps2; do
  echo "== $v"
  PMP_HIP_LIB=$L/libpmp_hip_$v.so timeout -k 10 200 python3 -u tools/lpa3d_probe.py 16 2>&1 | tail -3 || exit 1
done
