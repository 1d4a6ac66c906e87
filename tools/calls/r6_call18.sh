#!/bin/bash
# round 6, call 18: LPAStar3D per-query cycles against peak |U| (normal + PMP_STAMPS=2 builds)
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c18
PMP_PROBE_OUT=gpurun_out/r6c18/normal.npz timeout -k 10 200 python3 -u tools/lpa3d_probe.py 16 2>&1 | tail -2 || exit 1
PMP_PROBE_OUT=gpurun_out/r6c18/stamps2.npz PMP_HIP_LIB=$L/libpmp_hip_stamps2.so timeout -k 10 200 python3 -u tools/lpa3d_probe.py 16 2>&1 | tail -2 || exit 1
python3 tools/lpa3d_join.py gpurun_out/r6c18/normal.npz gpurun_out/r6c18/stamps2.npz
