#!/bin/bash
# round 5, call 8: Theta* / Lazy Theta* 2D parity on every engine at the current head; LPAStar3D issue
# breakdown (two SQ passes over the probe at 16 workers per CU)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c8
timeout -k 10 700 python -u -m pytest tests/test_graph_variants_gpu.py tests/test_rrt_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c8/tests.log 2>&1 || { tail -40 gpurun_out/c8/tests.log; exit 1; }
tail -1 gpurun_out/c8/tests.log
L=$R/python_motion_planning_amd
PMP_HIP_LIB=$L/libpmp_hip_rrtstamps.so timeout -k 10 200 python3 tools/rrt_time.py 4x16384 256x8192 > gpurun_out/c8/rrtstamps.log 2>&1 || { tail -20 gpurun_out/c8/rrtstamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c8/rrtstamps.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --legs rrt --detail-out gpurun_out/c8/rrt.json > gpurun_out/c8/rrt.out 2> gpurun_out/c8/rrt.err || { tail -20 gpurun_out/c8/rrt.err; exit 1; }
python3 -c "
import json; v=json.load(open('gpurun_out/c8/rrt.json'))['secondary']['rrt_star']; print('rrt', round(v['value']), 'kernel_ms', round(v['kernel_ms_per_launch'], 1))"
cd /tmp && export TMPDIR=/tmp
P1=SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD
P2=SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_INSTS_VMEM_WR,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_BUSY_CU_CYCLES,SQ_WAVE_CYCLES
i=0
for c in $P1 $P2; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc ${c//,/ } -d $R/gpurun_out/c8/lpa_p$i -o run -- python3 $R/tools/lpa3d_probe.py 16 > $R/gpurun_out/c8/lpa_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/c8/lpa_p$i.log; exit 1; }
  echo "pass $i"; python3 $R/tools/pmc_sum.py $R/gpurun_out/c8/lpa_p$i lpa3d_kernel
  rm -rf $R/gpurun_out/c8/lpa_p$i
done
