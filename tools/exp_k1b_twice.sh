R=$GRAFT_REPO_ROOT; cd /tmp && export TMPDIR=/tmp
UNIPEAK_LIB=$R/unipeak_amd/lib/libunipeak_hip_x2.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/x2 -o t -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/x2.log 2>&1 || exit 1
UNIPEAK_SIM_WORLD=8 UNIPEAK_LIB=$R/unipeak_amd/lib/libunipeak_hip_x2.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/x2s -o t -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $R/gpurun_out/x2s.log 2>&1 || exit 1
echo ok
