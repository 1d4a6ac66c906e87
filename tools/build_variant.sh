#!/bin/bash
# A/B builds: libpmp_hip_<name>.so with extra compile flags on the listed sources, the other objects
# shared with the default build (make first).  Run here (CPU container), not on the GPU box:
#   bash tools/build_variant.sh <name> "<-D flags>" astar2d_mq.hip [more.hip ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2; shift 2
C=$R/python_motion_planning_amd/csrc
OBJ=$R/build/obj
VO=$R/build/var_$NAME
mkdir -p $VO
make -s -C $C -j8
objs=()
for f in pmp_ctx astar2d astar2d_mq astar2d_sq astar3d dwa track rrt dstar dstar3d lpa lpa3d totp3d; do
  hit=0
  for s in "$@"; do [ "$s" = "$f.hip" ] && hit=1; done
  if [ $hit = 1 ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function $FLAGS -c -o $VO/$f.o $C/$f.hip
    objs+=($VO/$f.o)
  else
    objs+=($OBJ/$f.o)
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/python_motion_planning_amd/libpmp_hip_$NAME.so "${objs[@]}"
echo built libpmp_hip_$NAME.so
