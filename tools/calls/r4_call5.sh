#!/bin/bash
# round 4, call 5: unified kernel at <= 128 VGPRs (4 waves per SIMD): residency x tier-2 placement sweep
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/c5
for cfg in "uni2 48 12288 1" "uni3 48 12288 1" "uni3 56 14336 1" "uni3 64 16384 1" "uni3 64 16384 0" "uni3 56 14336 0"; do
  set -- $cfg
  PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_$1.so timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline --residency $2 --workers $3 --t2lds $4 > gpurun_out/c5/$1_$2_$4.json 2> gpurun_out/c5/$1_$2_$4.err || { tail -5 gpurun_out/c5/$1_$2_$4.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c5/$1_$2_$4.json').read().strip().splitlines()[-1]); print('$1 residency $2 t2lds $4', round(d['value']), round(d['ms_per_step']))"
done
