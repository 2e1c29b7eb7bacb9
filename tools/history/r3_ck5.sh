#!/bin/bash
# round 3 checkpoint 5: stencil march launch-mode probe across store-policy / priority variants
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r3_ck5_probe.jsonl; : > $out
timeout -k 10 200 python tools/sm_probe.py >> $out 2>gpurun_out/r3_ck5.err || exit $?
for v in smsc1 smnt smnoprio; do
  PCS_LIB_PATH=pycsou_amd/lib/var/$v/libpycsou_hip.so timeout -k 10 200 python tools/sm_probe.py >> $out 2>>gpurun_out/r3_ck5.err || exit $?
done
timeout -k 10 200 python tools/sm_probe.py >> $out 2>>gpurun_out/r3_ck5.err || exit $?
cat $out
