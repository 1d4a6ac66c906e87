#!/bin/bash
# round 5, call 4: DWA split hand-off without L2-writeback fences (stamps + timings), LPAStar3D bits
# in HBM (parity, plans/s, traffic), RRT* phase stamps, the A* headline half-block layout (parity,
# three alternating rounds vs the default, WRITE_SIZE of it and of its pop-store mirror)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c4
timeout -k 10 400 python -u -m pytest tests/test_dwa_gpu.py tests/test_lpastar3d_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c4/tests.log 2>&1 || { tail -40 gpurun_out/c4/tests.log; exit 1; }
tail -1 gpurun_out/c4/tests.log
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_blk2.so timeout -k 10 400 python -u -m pytest tests/test_astar2d_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c4/tests_blk2.log 2>&1 || { tail -40 gpurun_out/c4/tests_blk2.log; exit 1; }
tail -1 gpurun_out/c4/tests_blk2.log
timeout -k 10 200 python3 tools/dwa_split_probe.py > gpurun_out/c4/dwa_probe.log 2>&1 || { tail -20 gpurun_out/c4/dwa_probe.log; exit 1; }
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_dwastamps.so timeout -k 10 200 python3 tools/dwa_split_probe.py > gpurun_out/c4/dwa_stamps.log 2>&1 || { tail -20 gpurun_out/c4/dwa_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c4/dwa_probe.log; grep -E "ticks" gpurun_out/c4/dwa_stamps.log
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_rrtstamps.so timeout -k 10 200 python3 tools/rrt_time.py 4x16384 > gpurun_out/c4/rrt_stamps.log 2>&1 || { tail -20 gpurun_out/c4/rrt_stamps.log; exit 1; }
timeout -k 10 200 python3 tools/rrt_time.py 4x16384 256x4096 > gpurun_out/c4/rrt_time.log 2>&1 || { tail -20 gpurun_out/c4/rrt_time.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c4/rrt_stamps.log gpurun_out/c4/rrt_time.log
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --legs dyn3d --detail-out gpurun_out/c4/dyn3d.json > gpurun_out/c4/dyn3d.out 2>&1 || { tail -20 gpurun_out/c4/dyn3d.out; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/c4/dyn3d.json'))['secondary']
for k, v in d.items(): print(k, round(v['value']), 'kernel_ms', round(v['kernel_ms_per_launch'], 1))"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d $R/gpurun_out/c4/dyn3d_$c -o run -- python3 $R/bench.py --legs dyn3d --steps 1 --warmup 1 \
    --no-cpu-baseline --detail-out $R/gpurun_out/c4/dyn3d_$c.json > $R/gpurun_out/c4/dyn3d_$c.out 2>&1 || { echo "dyn3d $c failed"; tail -5 $R/gpurun_out/c4/dyn3d_$c.out; exit 1; }
done
python3 - $R/gpurun_out/c4 <<'PY'
import glob, sqlite3, sys
out = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    db = (glob.glob(f"{out}/dyn3d_{c}/**/*.db", recursive=True) + glob.glob(f"{out}/dyn3d_{c}/*.db"))[0]
    d = sqlite3.connect(db)
    cols = [r[1] for r in d.execute("pragma table_info(counters_collection)")]
    key = "dispatch_id" if "dispatch_id" in cols else "correlation_id"
    rows = list(d.execute(f"select kernel_name, sum(value) from counters_collection where counter_name = ? group by {key} order by {key}", (c,)))
    v = [x for n, x in rows if "lpa3d_kernel" in n]
    print(c, "lpa3d_kernel per-dispatch KiB", [round(x) for x in v])
PY
rm -rf $R/gpurun_out/c4/dyn3d_FETCH_SIZE $R/gpurun_out/c4/dyn3d_WRITE_SIZE
cd $R
for i in 1 2 3; do
  for v in default blk2; do
    lib=$R/python_motion_planning_amd/libpmp_hip.so
    [ "$v" = default ] || lib=$R/python_motion_planning_amd/libpmp_hip_$v.so
    PMP_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline --detail-out gpurun_out/c4/head_$v.json \
      > gpurun_out/c4/head_${v}_$i.out 2> gpurun_out/c4/head_${v}_$i.err || { tail -20 gpurun_out/c4/head_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/c4/head_${v}_$i.out').read().strip().splitlines()[-1]); print('headline $v', round(d['value']), 'ms/step', round(d['ms_per_step'], 1))"
  done
done
ATTR_DIR=attr4 SPECS="blk2:WRITE_SIZE,FETCH_SIZE blk2mir" bash tools/calls/r5_attr.sh
