#!/bin/bash
# gpu tests + A/B of staged record delivery
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/stage_tests.log 2>&1 || { tail -30 gpurun_out/stage_tests.log; exit 1; }
tail -3 gpurun_out/stage_tests.log
bash tools/stage_ab.sh
