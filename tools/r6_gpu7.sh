#!/bin/bash
# Round 6: plane lockstep of the 3-D update tiles -- A/B (PCS_3D_SYNC=0/1, alternating) on the four volume legs,
# the C5 centred update's read traffic with it, and the 3-D parity tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_7; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_pds.py -k "pds3d" tests/test_gpu_long2.py tests/test_gpu_determinism.py \
  > $O/tests.txt 2>&1 || { echo "tests failed"; grep -E "^E |FAILED" $O/tests.txt | head; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do for s in 0 1; do
  PCS_3D_SYNC=$s timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --legs "" --no-cpu-baseline \
     > $O/bench_s${s}_r$rep.txt 2> $O/bench_s${s}_r$rep.err || { echo "bench failed"; tail -5 $O/bench_s${s}_r$rep.err; exit 1; }
  python3 - $O/bench_s${s}_r$rep.txt $s <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split('\n')[-1])
print('sync', sys.argv[2], 'C3', d['value'], {k: (d[k]['it_per_s'], d[k]['roofline']['kernel_ms']) for k in ('volume_c4', 'volume_c5', 'volume_c4_cen', 'volume_c5_cen') if 'roofline' in (d.get(k) or {})})
PY
done; done
cd /tmp
PCS_PROBLEM=c4_cen PCS_DTYPE=f64 PCS_N=1024 PCS_ITERS=4 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$O/f -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/profile_step.py > $GRAFT_REPO_ROOT/$O/f.log 2>&1 || { echo "pmc f failed"; exit 1; }
PCS_PROBLEM=c4_cen PCS_DTYPE=f64 PCS_N=1024 PCS_ITERS=4 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/$O/w -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/profile_step.py > $GRAFT_REPO_ROOT/$O/w.log 2>&1 || { echo "pmc w failed"; exit 1; }
cd $GRAFT_REPO_ROOT
python3 tools/traffic_from_pmc.py $(find $O/f -name '*counter_collection.csv' | head -1) $(find $O/w -name '*counter_collection.csv' | head -1) $O/c5cen_traffic_sync.json k_pds3d_gen
find $O -name "*counter_collection.csv" -delete
echo ok
