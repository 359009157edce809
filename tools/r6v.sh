#!/bin/bash
# cold configs[1]: K1a stream priority high (default) vs normal; K3L vs wave-per-region at the rank
E="UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0"
REPS=2 tools/ab.sh "base|$E" "base|$E UNIPEAK_K1A_PRIO=0" | sed "s/UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0//"
