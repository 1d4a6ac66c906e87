# dev experiment: A* headline vs persistent workers per launch (LDS heap share per worker), 4 batches in flight
set -e
mkdir -p gpurun_out
: > gpurun_out/workers.log
for w in 2048 2560 3072 3328; do
  echo "workers=$w" >> gpurun_out/workers.log
  timeout -k 10 150 python -u bench.py --legs none --no-cpu-baseline --steps 20 --warmup 4 --workers $w >> gpurun_out/workers.log 2>&1
done
