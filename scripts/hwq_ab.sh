cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/hwq_$q.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/hwq_$q.json').read()); r=d['roofline']
print('hwq $q value %.4g ms/step %.3f expand %.3f alone %.3f' % (d['value'], d['ms_per_step'], r['kernel_ms'], r['alone']['kernel_ms']), {k: round(v, 3) for k, v in d['phases_ms'].items() if v})"
done; done
