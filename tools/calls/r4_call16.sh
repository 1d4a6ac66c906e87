#!/bin/bash
# round 4, call 16: the full GPU suite, smoke() and the driver's bench command at the head
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/c16
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/c16/gputest.log 2>&1 || { tail -40 gpurun_out/c16/gputest.log; exit 1; }
tail -2 gpurun_out/c16/gputest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/c16/smoke.log 2>&1 || { tail -20 gpurun_out/c16/smoke.log; exit 1; }
tail -1 gpurun_out/c16/smoke.log
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/c16/bench.jsonl 2> gpurun_out/c16/bench.err || { tail -20 gpurun_out/c16/bench.err; exit 1; }
tail -c 600 gpurun_out/c16/bench.jsonl
# 3D A* residency sweep (C5, the astar3d leg alone)
for res in 24 20 28 32; do
  timeout -k 10 200 python3 bench.py --legs astar3d --no-cpu-baseline --steps 1 --warmup 1 --a3-residency $res > gpurun_out/c16/a3_$res.json 2> gpurun_out/c16/a3_$res.err || { tail -5 gpurun_out/c16/a3_$res.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c16/a3_$res.json').read().strip().splitlines()[-1]); print('a3 residency $res', d['secondary']['astar3d'])"
done
