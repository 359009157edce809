#!/bin/bash
# A/B of variant builds (UNIPEAK_LIB suffixes as arguments) on one bench workload
# usage: WL=hg19-nondir1 bash tools/nd_ab.sh _a _b _a _b
R=$GRAFT_REPO_ROOT
WL=${WL:-hg19-nondir1}
for v in "$@"; do
  UNIPEAK_LIB=$R/unipeak_amd/lib/libunipeak_hip$v.so timeout -k 10 200 python $R/bench.py --no-cpu-baseline --workload $WL > $R/gpurun_out/wl$v.json 2>/dev/null || exit 1
  echo "$WL $v $(python $R/tools/jsum.py $R/gpurun_out/wl$v.json)"
done
