#!/bin/bash
# round 4, call 17: the round profile's kernel-trace pass (the default bench command under rocprofv3)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
ROUND=r4 PASSES=kt bash tools/profile_round.sh || exit 1
tail -c 400 gpurun_out/bench_prof.json
