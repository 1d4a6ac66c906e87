#!/bin/bash
# round 6, call 12: the whole headline batch (4096 pairs x 20, one launch) with its K longest queries
# (octile) on the single-query engine on a second stream beside the multi-query launch
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c12
for K in 64 128 256; do
  timeout -k 10 300 python3 bench.py --strong-share 0/1 --steps 20 --tail-sq $K > gpurun_out/c12/share_$K.out 2> gpurun_out/c12/share_$K.err || { tail -20 gpurun_out/c12/share_$K.err; exit 1; }
  tail -1 gpurun_out/c12/share_$K.out
done
