#!/bin/bash
# End-to-end CLI timing on one box: synthetic hg19 wig (tests/make_wig.py),
# then bin/regions with UNIPEAK_TIMING phases (parallel and serial ingest)
# and the oracle CLI restatement (1 core) on the same file.
set -e
D=${1:-gpurun_out/e2e}
mkdir -p "$D" /tmp/e2e
timeout -k 10 300 python -m tests.make_wig /tmp/e2e --table hg19 --samples 1 2> "$D/make.log"
ls -la /tmp/e2e >> "$D/make.log"
cd /tmp/e2e
for run in 1 2 3; do
  UNIPEAK_TIMING=1 timeout -k 10 300 "$GRAFT_REPO_ROOT/bin/regions" -f -c contigs.txt -o r_gpu.txt s0.wig 2> "$GRAFT_REPO_ROOT/$D/gpu_$run.err"
done
UNIPEAK_SERIAL_INGEST=1 UNIPEAK_TIMING=1 timeout -k 10 300 "$GRAFT_REPO_ROOT/bin/regions" -f -c contigs.txt -o r_ser.txt s0.wig 2> "$GRAFT_REPO_ROOT/$D/serial.err"
S=$(date +%s%N)
timeout -k 10 600 "$GRAFT_REPO_ROOT/oracle/_build/orc" regions -f -c contigs.txt -o r_orc.txt s0.wig 2> "$GRAFT_REPO_ROOT/$D/orc.err"
E=$(date +%s%N)
echo "orc_wall_ms $(( (E - S) / 1000000 ))" >> "$GRAFT_REPO_ROOT/$D/orc.err"
cmp r_gpu.txt r_orc.txt && echo "tables identical" >> "$GRAFT_REPO_ROOT/$D/orc.err"
cmp r_ser.txt r_orc.txt && echo "serial table identical" >> "$GRAFT_REPO_ROOT/$D/orc.err"
wc -l r_gpu.txt >> "$GRAFT_REPO_ROOT/$D/orc.err"
rm -rf /tmp/e2e
