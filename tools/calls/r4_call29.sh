#!/bin/bash
# round 4, call 29: 3D A* residency with the batch store (16 / 18 / 20 / 22 per CU), same box
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c29
for i in 1 2; do
for res in 20 16 18 22; do
  timeout -k 10 200 python3 bench.py --legs astar3d --no-cpu-baseline --steps 1 --warmup 1 --a3-residency $res > gpurun_out/c29/r${res}_$i.json 2> gpurun_out/c29/r${res}_$i.err || { tail -5 gpurun_out/c29/r${res}_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c29/r${res}_$i.json').read().strip().splitlines()[-1]); print('a3 residency $res', d['secondary']['astar3d']['value'])"
done
done
