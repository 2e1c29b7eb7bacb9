#!/bin/bash
# round 3 checkpoint 19: rehearsal of bench.py's N = 2 path on the one-GPU box (gloo transport,
# both ranks on GPU 0): the slab C3 line, the C4 / C4-centred volume legs (smaller volumes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PCS_BENCH_BACKEND=gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 20 --warmup 4 --size 2048 --volumes "c4:256:f32:4,c4_cen:256:f32:4:centered" > gpurun_out/r3_ck19.json 2> gpurun_out/r3_ck19.err || { tail -30 gpurun_out/r3_ck19.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r3_ck19.json').read().splitlines()[-1])
print({k: d[k] for k in ('value','n_gpus','ms_per_step','loop','loop_fallback') if k in d}); print(d['config']['workload'][:200])
for k in ('volume_c4','volume_c4_cen'): print(k, {q: d[k].get(q) for q in ('it_per_s','error','banded_order','halo_bytes_per_side_per_iter')})"
