#!/bin/bash
# C5 voice-clone bench lines (batch 8 and 1) next to the plain batch-8 line
set -eo pipefail
O=gpurun_out/${1:-r01az}; mkdir -p $O
timeout -k 10 300 python bench.py --voice-clone --batch 8 --no-cpu-baseline > $O/vc_b8.json 2> $O/vc_b8.err
timeout -k 10 300 python bench.py --voice-clone --batch 1 --no-cpu-baseline > $O/vc_b1.json 2> $O/vc_b1.err
timeout -k 10 300 python bench.py --batch 8 --no-cpu-baseline --no-profile > $O/b8.json 2> $O/b8.err
echo done
