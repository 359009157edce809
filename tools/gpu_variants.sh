#!/bin/bash
# Same-box comparison of whole source trees (git worktrees under exp/, each
# with its own built library, or "." for this tree): per tree a bench line
# (isolated per-kernel times) and one rocprofv3 SQ counter pass.
# usage: TAG=bisect tools/gpu_variants.sh . exp/wt_<commit> lib:NAME ...
# (lib:NAME = this tree with UNIPEAK_LIB=unipeak_amd/lib/libunipeak_hip_NAME.so;
#  env:NAME:VAR=VALUE = this tree with VAR=VALUE in the environment)
# Results: gpurun_out/$TAG/<name>.json, <name>_sq/ (counter csv).
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${TAG:-variants}; mkdir -p "$F"
WL=${WORKLOAD:-hg19-dir1}
SQ=${SQ:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM"}
for rep in $(seq 1 "${REPS:-1}"); do
for v in "$@"; do
  unset UNIPEAK_LIB; [ -n "$ENVSET" ] && unset "${ENVSET%%=*}"; ENVSET=
  case "$v" in
    lib:*) n=${v#lib:}; export UNIPEAK_LIB=$R/unipeak_amd/lib/libunipeak_hip_$n.so; v=. ;;
    env:*) n=${v#env:}; ENVSET=${n#*:}; n=${n%%:*}; export "$ENVSET"; v=. ;;
    *) n=$(basename "$(cd "$R/$v" && pwd)"); [ "$v" = . ] && n=head ;;
  esac
  cd "$R/$v" || exit 1
  timeout -k 10 200 python bench.py --workload $WL --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline \
    > "$F/${n}_r$rep.json" 2> "$F/${n}_r$rep.err" || { tail -3 "$F/${n}_r$rep.err"; exit 1; }
  echo "$n r$rep: $(cut -c1-120 "$F/${n}_r$rep.json")"
  python - "$F/${n}_r$rep.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r = d["roofline"]
print("   ", d["ms_per_step"], "k1a", r["kernel_ms"], "iso", r.get("isolated_ms"))
EOF
  if [ "$rep" = 1 ] && [ -z "$NO_SQ" ]; then
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv \
      -d "$F/${n}_sq" -o p -- python3 "$R/$v/bench.py" --workload $WL --steps 3 --warmup 1 --no-cpu-baseline \
      > "$F/${n}_sq.log" 2>&1) || { tail -3 "$F/${n}_sq.log"; exit 1; }
  fi
done
done
echo variants-ok
