set -o pipefail
mkdir -p gpurun_out/nrm1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "sep_ata" tests/test_gpu_pds.py::test_pds3d_ata_opt_in_matches_reference > gpurun_out/nrm1/tests.txt 2>&1 && \
timeout -k 10 180 python3 tools/ata_probe.py > gpurun_out/nrm1/probe.txt 2>&1
rc=$?; tail -5 gpurun_out/nrm1/tests.txt; cat gpurun_out/nrm1/probe.txt; exit $rc
