# dev experiment: A* headline vs batches in flight (one stream + scratch context each)
set -e
mkdir -p gpurun_out
: > gpurun_out/streams.log
for s in ${STREAMS:-4 6 4 6}; do
  echo "streams=$s" >> gpurun_out/streams.log
  timeout -k 10 200 python -u bench.py --legs none --no-cpu-baseline --steps 12 --warmup 6 --streams $s >> gpurun_out/streams.log 2>&1
done
