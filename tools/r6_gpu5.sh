#!/bin/bash
# Round 6: C5 at its real size (fused vs generic, both K kinds), the deep-halo probe with its kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_5; mkdir -p $O
true || \
  > $O/c5.txt 2>&1 || { echo "c5 test failed"; grep -E "^E |FAILED|Error" $O/c5.txt | head -30; tail -5 $O/c5.txt; exit 1; }
tail -3 $O/c5.txt
timeout -k 10 300 python -u tools/deep_probe.py > $O/deep_probe.jsonl 2> $O/deep_probe.err || { echo "probe failed"; tail -20 $O/deep_probe.err; exit 1; }
cat $O/deep_probe.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/deep_probe.py > $O/deep_probe_prof.log 2>&1 || { echo "prof failed"; tail -5 $O/deep_probe_prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/deep_probe_kernel_stats.csv \;
find $O/prof -name "*kernel_trace.csv" -delete
echo ok
