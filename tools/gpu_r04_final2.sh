#!/bin/bash
# round-4 closing set on the final build: part A then part B
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; cd "$R" || exit 1
tools/gpu_r04_final_a.sh ${1:-final2}_a && tools/gpu_r04_final_b.sh ${1:-final2}_b
