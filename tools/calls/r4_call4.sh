#!/bin/bash
# round 4, call 4: unified kernel residency sweep; strong-scaling legs at world 1; full default bench
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/c4
U=$R/python_motion_planning_amd/libpmp_hip_uni.so
for cfg in "32 8192" "40 10240" "48 12288"; do
  set -- $cfg
  PMP_HIP_LIB=$U timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline --residency $1 --workers $2 > gpurun_out/c4/uni_res$1.json 2> gpurun_out/c4/uni_res$1.err || { tail -5 gpurun_out/c4/uni_res$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c4/uni_res$1.json').read().strip().splitlines()[-1]); print('uni residency $1', round(d['value']), round(d['ms_per_step']))"
done
timeout -k 10 400 python3 bench.py --scaling strong --legs dwa,astar3d,lqr,mpc --no-cpu-baseline --steps 2 --warmup 1 --detail-out gpurun_out/c4/strong_detail.json > gpurun_out/c4/strong.json 2> gpurun_out/c4/strong.err || { tail -5 gpurun_out/c4/strong.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/c4/strong_detail.json'))
for k in ('mpc_sampled_dwa','astar3d','lqr','mpc_qp'):
    print(k, d['secondary'][k].get('scaling'), d['secondary'][k].get('strong_scaling_gather'), round(d['secondary'][k]['value']))
"
timeout -k 10 500 python3 bench.py --detail-out gpurun_out/c4/full_detail.json > gpurun_out/c4/full.json 2> gpurun_out/c4/full.err || { tail -5 gpurun_out/c4/full.err; exit 1; }
tail -c 3000 gpurun_out/c4/full.json
