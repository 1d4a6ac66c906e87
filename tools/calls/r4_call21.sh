#!/bin/bash
# round 4, calls 21 / 24 / 31 (final head): the full GPU suite, smoke(), the driver's bench command, then the
# round profile's kernel-trace pass
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/c21
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c21/gputest.log 2>&1 || { tail -40 gpurun_out/c21/gputest.log; exit 1; }
tail -2 gpurun_out/c21/gputest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/c21/smoke.log 2>&1 || { tail -20 gpurun_out/c21/smoke.log; exit 1; }
tail -1 gpurun_out/c21/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/c21/bench.jsonl 2> gpurun_out/c21/bench.err || { tail -20 gpurun_out/c21/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/c21/bench.jsonl').read().strip().splitlines()[-1]); print(round(d['value']), {k: v['value'] for k, v in d['secondary'].items()})"
ROUND=r4 PASSES=kt bash tools/profile_round.sh || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/bench_prof.json').read().strip().splitlines()[-1]); print('under rocprof', round(d['value']), d['ms_per_step'])"
