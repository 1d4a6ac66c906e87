#!/bin/bash
# DWA kernel variants (threads per agent) on the GPU box: parity tests with the default build, the
# bench's control leg per variant, and FETCH_SIZE / WRITE_SIZE passes of the default build.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/dwa
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_dwa_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/test.log 2>&1
for L in libpmp_hip.so libpmp_hip_dwa768.so libpmp_hip_dwa512.so; do
  PMP_HIP_LIB=$R/python_motion_planning_amd/$L timeout -k 10 200 python3 bench.py --legs dwa --steps 1 --warmup 1 \
    --no-cpu-baseline --control-steps 20 > $OUT/bench_$L.json 2> $OUT/bench_$L.err
  python3 -c "import json; d=json.loads(open('$OUT/bench_$L.json').read().strip().splitlines()[-1])['secondary']['mpc_sampled_dwa']; print('$L', round(d['value']), d['kernel_ms_per_launch'])"
done
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d $OUT/prof_$C -o run -- python3 $R/bench.py --legs dwa --steps 1 --warmup 1 \
    --no-cpu-baseline --control-steps 3 > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err
done
echo dwa-ab-done
