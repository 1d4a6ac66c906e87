#!/bin/bash
# round 5, call 21: Theta* / Lazy Theta* 2D residency sweep on the shared context; the new RRT bins
# edge-case parity test
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c21
timeout -k 10 300 python -u -m pytest tests/test_rrt_gpu.py -x -q -k bins --timeout 200 --timeout-method thread > gpurun_out/c21/tests.log 2>&1 || { tail -30 gpurun_out/c21/tests.log; exit 1; }
tail -1 gpurun_out/c21/tests.log
theta() {  # name args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --legs graphs --no-cpu-baseline --detail-out gpurun_out/c21/$n.json "$@" \
    > gpurun_out/c21/$n.out 2> gpurun_out/c21/$n.err || { tail -20 gpurun_out/c21/$n.err; return 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c21/$n.json'))['secondary']
for k in ('theta_star_2d', 'lazy_theta_star_2d'): print('$n', k, round(d[k]['value']), 'kernel_ms', round(d[k]['kernel_ms_per_launch']))"
}
for r in 24 40 48 32; do
  theta r$r --theta-residency $r || exit 1
done
