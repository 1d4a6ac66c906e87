# dev experiment: RRT* leg vs batches in flight / queries per launch
set -e
mkdir -p gpurun_out
: > gpurun_out/rrt.log
for cfg in "3 256" "4 256" "6 256" "3 512"; do
  set -- $cfg
  echo "streams=$1 queries=$2" >> gpurun_out/rrt.log
  timeout -k 10 300 python -u bench.py --legs rrt --no-cpu-baseline --steps 1 --warmup 1 --rrt-streams $1 --rrt-queries $2 --rrt-steps 8 >> gpurun_out/rrt.log 2>&1
done
