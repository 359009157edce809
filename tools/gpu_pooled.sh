set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_plane.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt_pooled.log 2>&1; r=$?; tail -3 gpurun_out/pyt_pooled.log; grep -E "FAILED|Error|assert" gpurun_out/pyt_pooled.log | head; [ $r = 0 ] || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pyt_pooledfull.log 2>&1; r=$?; tail -2 gpurun_out/pyt_pooledfull.log; grep -E "FAILED|Error" gpurun_out/pyt_pooledfull.log | head -5; [ $r = 0 ] || exit 1
mkdir -p gpurun_out/pooled
for w in hg19-dir1 hg19-nondir1 hg19-8s1c; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/pooled/$w.json 2> gpurun_out/pooled/$w.err || { tail -3 gpurun_out/pooled/$w.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/pooled/$w.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$w', d['value'], d['ms_per_step'], 'k1a', r['kernel_ms'], 'iso', r['isolated_ms'])"
done
timeout -k 10 400 python bench.py --workload hg19mm9-32rep --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pooled/rep.json 2> gpurun_out/pooled/rep.err || { tail -3 gpurun_out/pooled/rep.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/pooled/rep.json').read().strip().splitlines()[-1]); r=d['roofline']
print('32rep', d['value'], d['ms_per_step'], 'k1a', r['kernel_ms'], 'iso', r['isolated_ms'], d['regions'])"
