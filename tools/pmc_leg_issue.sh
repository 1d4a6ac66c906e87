#!/bin/bash
# PMC issue breakdown (2 passes of 8 SQ counters) of one kernel in one bench leg:
#   bash tools/pmc_leg_issue.sh <leg> <kernel-substring> <tag> [extra bench args]
R=${GRAFT_REPO_ROOT:-/root/repo}
LEG=$1; KER=$2; TAG=$3; shift 3; EXTRA="$@"
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
S1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY"
S2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES"
i=0
for set in "$S1" "$S2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set -d $OUT/p$i -o run -- python3 $R/bench.py --legs $LEG --no-cpu-baseline --steps 1 --warmup 1 $EXTRA > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT $KER <<'PY'
import glob, sqlite3, sys
out, ker = sys.argv[1], sys.argv[2]
vals = {}
for db in sorted(glob.glob(f"{out}/p*/**/*.db", recursive=True)):
    d = sqlite3.connect(db)
    for name, s in d.execute("select counter_name, sum(value) from counters_collection where kernel_name like ? group by counter_name", (f"%{ker}%",)):
        vals[name] = s
wc = vals.get("SQ_WAVE_CYCLES", 1)
for k, v in sorted(vals.items()):
    print(f"  {k:24s} {v:18.0f}  per-wave-cycle {v / wc:.3f}")
PY
rm -rf $OUT/p1 $OUT/p2
