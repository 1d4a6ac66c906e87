#!/bin/bash
# round 6, call 48: D* in two passes (first pass W*H + 64 entries per query, the overflowing queries
# re-run at the bound) -- D* tests, the probe, the D* legs
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/r6c48
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_dstar_gpu.py \
  > gpurun_out/r6c48/pytest.log 2>&1 || { tail -30 gpurun_out/r6c48/pytest.log; exit 1; }
tail -1 gpurun_out/r6c48/pytest.log
timeout -k 10 300 python3 -u tools/dstar_cap_probe.py || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --legs dstar --steps 1 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r6c48/b_$r.out 2> gpurun_out/r6c48/b_$r.err || { tail -20 gpurun_out/r6c48/b_$r.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r6c48/b_$r.out').read().strip().splitlines()[-1]); print('round $r', d['secondary']['dstar_256']['value'], d['secondary']['dstar_512']['value'])"
done
