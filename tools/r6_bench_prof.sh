#!/bin/bash
# Round 6: the driver's bench command, plain and under rocprofv3 --kernel-trace --stats (the summary the
# headline roofline is checked against)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${R6_OUT:-r6_bench}; mkdir -p $O
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/bench_prof.err || { echo "prof failed"; tail -5 $O/bench_prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/bench_kernel_stats.csv \;
find $O/prof -name "*kernel_trace.csv" -delete
echo ok
