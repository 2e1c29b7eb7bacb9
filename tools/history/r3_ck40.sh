#!/bin/bash
# round 3 checkpoint 40: full checkpoint (GPU tests, smoke, bench, kernel stats), then the C5 ATA A/B
set -o pipefail
bash tools/ck_run.sh r3_ck40 && bash tools/r3_ck41.sh
