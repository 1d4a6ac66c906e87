#!/bin/bash
# round 5, call 3: DWA split phase stamps + timings after the LDS leaf-sum staging; the A* headline
# write attribution (mirror builds, tools/calls/r5_attr.sh); LPAStar3D FETCH / WRITE passes
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c3
timeout -k 10 300 python -u -m pytest tests/test_dwa_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c3/dwa_tests.log 2>&1 || { tail -40 gpurun_out/c3/dwa_tests.log; exit 1; }
tail -1 gpurun_out/c3/dwa_tests.log
timeout -k 10 200 python3 tools/dwa_split_probe.py > gpurun_out/c3/dwa_probe.log 2>&1 || { tail -20 gpurun_out/c3/dwa_probe.log; exit 1; }
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_dwastamps.so timeout -k 10 200 python3 tools/dwa_split_probe.py > gpurun_out/c3/dwa_stamps.log 2>&1 || { tail -20 gpurun_out/c3/dwa_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c3/dwa_probe.log gpurun_out/c3/dwa_stamps.log
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d $R/gpurun_out/c3/dyn3d_$c -o run -- python3 $R/bench.py --legs dyn3d --steps 1 --warmup 1 \
    --no-cpu-baseline --detail-out $R/gpurun_out/c3/dyn3d_$c.json > $R/gpurun_out/c3/dyn3d_$c.out 2>&1 || { echo "dyn3d $c failed"; tail -5 $R/gpurun_out/c3/dyn3d_$c.out; exit 1; }
done
python3 - $R/gpurun_out/c3 <<'PY'
import glob, sqlite3, sys, json
out = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    db = (glob.glob(f"{out}/dyn3d_{c}/**/*.db", recursive=True) + glob.glob(f"{out}/dyn3d_{c}/*.db"))[0]
    d = sqlite3.connect(db)
    cols = [r[1] for r in d.execute("pragma table_info(counters_collection)")]
    key = "dispatch_id" if "dispatch_id" in cols else "correlation_id"
    rows = list(d.execute(f"select kernel_name, sum(value) from counters_collection where counter_name = ? group by {key} order by {key}", (c,)))
    for k in ("lpa3d_kernel", "dstar3d_kernel"):
        v = [x for n, x in rows if k in n]
        print(c, k, "per-dispatch KiB", [round(x) for x in v])
PY
rm -rf $R/gpurun_out/c3/dyn3d_FETCH_SIZE $R/gpurun_out/c3/dyn3d_WRITE_SIZE
cd $R && SPECS="default:WRITE_SIZE,FETCH_SIZE mir1 mir2 mir4 mir8" bash tools/calls/r5_attr.sh
