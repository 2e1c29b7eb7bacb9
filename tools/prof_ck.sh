set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2ck5
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r2ck5/prof -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r2ck5/prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r2ck5/prof.log; exit 3; }
find gpurun_out/r2ck5/prof \( -name '*kernel_trace.csv' -o -name '*agent_info.csv' \) -delete
find gpurun_out/r2ck5 -type f | head
