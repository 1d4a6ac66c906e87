# dev experiment: A* headline vs batches in flight (streams), HIP hardware queues and workers
set -e
mkdir -p gpurun_out
: > gpurun_out/streams3.log
for cfg in "4 3 3072" "8 3 3072" "8 4 3072" "8 5 3072" "8 4 2560" "8 5 2560"; do
  set -- $cfg
  echo "hwq=$1 streams=$2 workers=$3" >> gpurun_out/streams3.log
  GPU_MAX_HW_QUEUES=$1 timeout -k 10 150 python -u bench.py --legs none --no-cpu-baseline --steps 20 --warmup $2 --streams $2 --workers $3 >> gpurun_out/streams3.log 2>&1
done
