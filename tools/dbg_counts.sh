R="${GRAFT_REPO_ROOT:?}"
for v in dbg dbgint; do
UNIPEAK_DEBUG_COUNTS=1 UNIPEAK_LIB=$R/unipeak_amd/lib/libunipeak_hip_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/$v.json 2> gpurun_out/$v.err || exit 1
echo $v; grep "K1 strips" gpurun_out/$v.err | tail -1
done
