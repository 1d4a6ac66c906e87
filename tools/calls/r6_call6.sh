#!/bin/bash
# round 6, call 6: every-launch checks of the DWA / LQR / MPC legs; the C2 strong-split share (rank 0
# of 8) on one GPU, all on the multi-query engine vs its longest queries on the single-query engine
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c6
timeout -k 10 400 python3 bench.py --legs dwa,lqr,mpc --steps 2 --warmup 1 --no-cpu-baseline \
  --detail-out gpurun_out/c6/legs.json > gpurun_out/c6/legs.out 2> gpurun_out/c6/legs.err || { tail -20 gpurun_out/c6/legs.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/c6/legs.json'))
for k, v in d['secondary'].items(): print(k, v['value'], 'checked', v.get('timed_launches_checked'))"
for K in 256 512; do
  timeout -k 10 300 python3 bench.py --strong-share 0/8 --steps 20 --tail-sq $K > gpurun_out/c6/share_$K.out 2> gpurun_out/c6/share_$K.err || { tail -20 gpurun_out/c6/share_$K.err; exit 1; }
  tail -1 gpurun_out/c6/share_$K.out
done
