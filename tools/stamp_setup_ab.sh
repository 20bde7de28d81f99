#!/bin/bash
# same-box: the stamp slots set up before the timed region (default) or only after it
set -u
cd "$(dirname "$0")/.."
p=29580
j() { python3 - "$1" /root/repo/gpurun_out/c5ab.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][0]); c = d["config"]
print(sys.argv[1], round(d["ms_per_step"], 4), json.dumps(c.get("time_split_s")))
PY
}
for r in 1 2; do
  for v in setup none; do
    p=$((p+1)); t=0; [ $v = none ] && t=1
    MAXCOVER_BENCH_NO_STAMP_SETUP=$t MAXCOVER_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
       --master-addr 127.0.0.1 --master-port $p bench.py --gpus 2 --config 5 --no-cpu --dist-backend gloo \
       --steps 2 --warmup 1 --mads-mode shard > /root/repo/gpurun_out/c5ab.log 2>&1 || exit $?
    j "c5x2 $v"
    MAXCOVER_BENCH_NO_STAMP_SETUP=$t timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu > /root/repo/gpurun_out/c5ab.log 2>&1 || exit $?
    j "c5 $v"
    MAXCOVER_BENCH_NO_STAMP_SETUP=$t timeout -k 10 300 python bench.py --no-cpu --no-extras --steps 40 > /root/repo/gpurun_out/c5ab.log 2>&1 || exit $?
    j "c4 $v"
    p=$((p+1))
    MAXCOVER_BENCH_NO_STAMP_SETUP=$t MAXCOVER_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --no-cpu --no-extras --dist-backend gloo --steps 20 > /root/repo/gpurun_out/c5ab.log 2>&1 || exit $?
    j "c4x2 $v"
  done
done
