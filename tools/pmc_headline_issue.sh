#!/bin/bash
# PMC issue breakdown of the A* 2D multi-query kernel at the headline geometry (W_=15360 groups, RES=60
# queries resident per CU, tier-2 bits in LDS), REPEAT batches of the C2 queries in one launch
# (tools/astar2d_probe.py); MODE=c1 ENGINE=3 KERN=sq: the single-query engine on the README query.
# Usage: [LIB=libpmp_hip_x.so] bash tools/pmc_headline_issue.sh tag
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-head}
OUT=$R/gpurun_out/pmc_issue_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ -n "$LIB" ] && export PMP_HIP_LIB=$R/python_motion_planning_amd/$LIB
S1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY"
S2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_CYCLES"
i=0
for set in "$S1" "$S2"; do
  i=$((i+1))
  ENGINE=${ENGINE:-1} T2LDS=1 WORKERS=${W_:-15360} RESIDENCY=${RES:-60} MODE=${MODE:-batch} REPEAT=${REPEAT:-4} REPS=1 timeout -s KILL 150 rocprofv3 --pmc $set -d $OUT/p$i -o run -- python3 $R/tools/astar2d_probe.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT ${KERN:-mq} <<'PY'
import glob, re, sqlite3, sys
out, kern = sys.argv[1], sys.argv[2]
vals = {}
for db in sorted(glob.glob(f"{out}/p*/**/*.db", recursive=True)):
    d = sqlite3.connect(db)
    for name, s in d.execute("select counter_name, sum(value) from counters_collection where kernel_name like ? group by counter_name", (f"%{kern}%",)):
        vals[name] = s
m = re.search(r"\((\d+) plans/s\).*pushes (\d+) pops (\d+) exp (\d+)", open(f"{out}/p1.log").read())
pl, P, Q, E = map(int, m.groups())
print(f"plans/s {pl} ops {P + Q} expansions {E}")
for k, v in sorted(vals.items()):
    print(f"  {k:24s} {v:18.0f}  per-op {v / (P + Q):9.2f}  per-wave-cycle {v / vals.get('SQ_WAVE_CYCLES', 1):.3f}")
PY
