#!/bin/bash
# Dev loop on the GPU box: the given GPU test files, then the given bench legs (one timed step each,
# no CPU baseline), printing each leg's value and roofline fraction.
# usage: TESTS="tests/test_x.py ..." LEGS=dstar,dyn3d OUT=name bash tools/leg_check.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
O=gpurun_out/${OUT:-check}
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest $TESTS -x -q --timeout 250 --timeout-method thread > $O.test.log 2>&1
  rc=$?; tail -2 $O.test.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$LEGS" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py --legs $LEGS --no-cpu-baseline --steps ${STEPS:-1} --warmup 1 \
      --detail-out $O.detail.json $BENCH_ARGS > $O.bench.json 2> $O.bench.err || { tail -5 $O.bench.err; exit 1; }
  python3 - "$O.bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", d["value"], d["roofline"].get("frac"))
for k, v in d["secondary"].items():
    print(k, v["value"], v.get("frac"))
PY
fi
