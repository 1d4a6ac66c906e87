#!/bin/bash
# round 5, call 1: the GPU suite (RRT* coarse tree in LDS, DWA k-split, LPA* U past the LDS share, geometry restore, the 3D
# kernel without the decrease-key variant), the DWA 32-agent step time, the MPC tolerance probe, then
# the A* 2D write attribution (tools/r5_attr.sh)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/c1/gpu_tests.log 2>&1 || { tail -60 gpurun_out/c1/gpu_tests.log; exit 1; }
tail -3 gpurun_out/c1/gpu_tests.log
for na in 32 256; do
  timeout -k 10 200 python3 bench.py --legs dwa --agents $na --steps 2 --warmup 1 --no-cpu-baseline --control-steps 50 \
    --detail-out gpurun_out/c1/dwa_$na.json > gpurun_out/c1/dwa_$na.out 2> gpurun_out/c1/dwa_$na.err || { tail -20 gpurun_out/c1/dwa_$na.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c1/dwa_$na.json'))['secondary']['mpc_sampled_dwa']; print('dwa agents $na', d['value'], 'kernel ms', d['kernel_ms_per_launch'], d.get('timed_launches_checked'))"
done
timeout -k 10 300 python3 bench.py --legs rrt --steps 2 --warmup 1 --no-cpu-baseline --rrt-steps 3 \
  --detail-out gpurun_out/c1/rrt.json > gpurun_out/c1/rrt.out 2> gpurun_out/c1/rrt.err || { tail -20 gpurun_out/c1/rrt.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c1/rrt.json'))['secondary']['rrt_star']; print('rrt*', d['value'], 'kernel ms', d['kernel_ms_per_launch'], d.get('timed_launches_checked'), d['roofline']['frac'])"
timeout -k 10 200 python3 tools/mpc_tol.py > gpurun_out/c1/mpc_tol.log 2>&1 || { tail -20 gpurun_out/c1/mpc_tol.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c1/mpc_tol.log
bash tools/r5_attr.sh
