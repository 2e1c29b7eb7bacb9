# k_sep2d_nrm: parity subset, then the probe on the default build and the given variants
set -o pipefail
mkdir -p gpurun_out/nrm1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py -k "sep_ata" tests/test_gpu_pds.py::test_pds3d_ata_opt_in_matches_reference > gpurun_out/nrm1/tests.txt 2>&1 || { tail -30 gpurun_out/nrm1/tests.txt; exit 1; }
tail -2 gpurun_out/nrm1/tests.txt
bash tools/nrm_ablate.sh "$@"
