#!/bin/bash
# round 6, call 7: PMC of the headline launch, round-5 build vs new (tools/ab_headline.py, one build per
# process, 5-batch warmup + one 20-batch launch): FETCH_SIZE, WRITE_SIZE and the SQ issue counters
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/c7
for lib in base new; do
  so=$L/libpmp_hip.so; [ $lib = base ] && so=$L/libpmp_hip_base.so
  for pass in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
    tag=$(echo $pass | cut -d' ' -f1)
    timeout -k 10 300 rocprofv3 --pmc $pass -d $R/gpurun_out/c7/${lib}_$tag -o run -- python3 $R/tools/ab_headline.py $so --rounds 1 --reps 1 \
      > $R/gpurun_out/c7/${lib}_$tag.log 2>&1 || { tail -20 $R/gpurun_out/c7/${lib}_$tag.log; exit 1; }
    python3 - <<PY
import sqlite3, glob
p = glob.glob("$R/gpurun_out/c7/${lib}_$tag/**/*.db", recursive=True) + glob.glob("$R/gpurun_out/c7/${lib}_$tag/*.db")
d = sqlite3.connect(p[0])
rows = list(d.execute("select dispatch_id, kernel_name, counter_name, sum(value) from counters_collection group by dispatch_id, counter_name order by dispatch_id"))
big = {}
for disp, name, cn, v in rows:
    if "astar2d_mqu_kernel" in name: big.setdefault(disp, {})[cn] = v
last = sorted(big)[-1]
print("$lib", "dispatch", last, {k: "%.4g" % v for k, v in big[last].items()})
PY
    rm -rf $R/gpurun_out/c7/${lib}_$tag
  done
done
