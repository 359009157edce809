#!/bin/bash
# nondirectional K3: batched LDS reads in the correlation sums (+ K3 at 4 waves/SIMD) vs the committed build
set -o pipefail
T=r6x; mkdir -p gpurun_out/$T
true
true
E="UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0"
WORKLOAD=hg19-nondir1 NO_SIM=1 REPS=2 tools/ab.sh "base|$E" "tb8|$E" | sed "s/UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0//"
