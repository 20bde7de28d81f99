set -u
mkdir -p gpurun_out/abs
for r in 1 2 3; do
  for v in timed separate; do
    timeout -k 10 120 python bench.py --no-cpu --no-extras --stamps $v > gpurun_out/abs/$v$r.log 2>&1 || exit $?
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/abs/$v$r.log') if l.startswith('{')][0])
print('$v', round(d['ms_per_step'],4), round(d['roofline']['chain_ms']*1e3,1), {k: round(x['avg_us'],1) for k,x in d['roofline']['kernels'].items()})"
  done
done
