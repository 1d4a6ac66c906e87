#!/bin/bash
# round 6, call 19: LPAStar3D extractPath cycle shortcut -- lpa3d parity (the stuck C5 query and its
# apply_change rounds against the oracle), the probe against the round-5 form, the bench's dyn3d leg
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c19
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lpastar3d_gpu.py \
  > gpurun_out/r6c19/pytest.log 2>&1 || { tail -30 gpurun_out/r6c19/pytest.log; exit 1; }
tail -1 gpurun_out/r6c19/pytest.log
for v in new old; do
  if [ $v = old ]; then export PMP_HIP_LIB=$L/libpmp_hip_l3old.so; else unset PMP_HIP_LIB; fi
  echo "== $v"
  timeout -k 10 200 python3 -u tools/lpa3d_probe.py 16 2>&1 | tail -2 | head -1 || exit 1
done
unset PMP_HIP_LIB
timeout -k 10 600 python3 bench.py --legs dyn3d --steps 3 --warmup 1 --detail-out gpurun_out/r6c19/detail.json \
  > gpurun_out/r6c19/bench.out 2> gpurun_out/r6c19/bench.err || { tail -20 gpurun_out/r6c19/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r6c19/detail.json'))
for k, v in d.items():
    if 'star3d' in k.lower() or 'dyn3d' in k.lower(): print(k, {a: v[a] for a in ('value', 'unit') if isinstance(v, dict) and a in v})
" || true
tail -1 gpurun_out/r6c19/bench.out | head -c 3000
