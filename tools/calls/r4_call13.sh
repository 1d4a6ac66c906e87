#!/bin/bash
# round 4, call 13: which kernel serves a lone query, and its dispatch time (rocprofv3 kernel trace)
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/c13
cd /tmp && export TMPDIR=/tmp
for m in c1 c2med; do
  for e in 0 3; do
    MODE=$m ENGINE=$e REPS=3 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c13/prof_${m}_$e -o run -- python3 $R/tools/astar2d_probe.py > $R/gpurun_out/c13/${m}_$e.log 2>&1 || { tail -20 $R/gpurun_out/c13/${m}_$e.log; exit 1; }
    grep -v amdgpu.ids $R/gpurun_out/c13/${m}_$e.log | grep plans
    f=$(find $R/gpurun_out/c13/prof_${m}_$e -name "*kernel_stats.csv" | head -1)
    grep -i astar $f | cut -c1-250; echo "--- $m $e"
  done
done
find $R/gpurun_out/c13 -name "*.db" -delete
