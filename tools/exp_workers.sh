# dev experiment: A* headline vs persistent workers per launch (LDS heap share per worker shrinks
# as workers per CU grow; the VGPR limit is 5 waves per SIMD = 20 per CU)
set -e
mkdir -p gpurun_out
: > gpurun_out/workers.log
for w in ${WORKERS:-3072 4096 5120}; do
  echo "workers=$w" >> gpurun_out/workers.log
  timeout -k 10 150 python -u bench.py --legs none --no-cpu-baseline --steps 12 --warmup 4 --workers $w >> gpurun_out/workers.log 2>&1
done
