set -o pipefail
for v in nowait lead8; do echo "== $v"; PCS_LIB_PATH=pycsou_amd/lib/var/$v/libpycsou_hip.so timeout -k 10 200 python -u tools/sync_probe.py 2>/dev/null | grep graph\":\ true || exit 1; done
