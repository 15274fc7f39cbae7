#!/bin/bash
# Lists every kernel instantiation with a non-zero scratch (spill / stack)
# size (development tool): an accidental spill or out-of-line call in a
# latency-bound kernel costs microseconds per launch.
#   bash tools/scratch_check.sh
cd "$(dirname "$0")/../qwen3-tts-c_amd" || exit 1
for f in csrc/hip/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -c "$f" -o /tmp/qtts_scratch_check.o \
      -Rpass-analysis=kernel-resource-usage 2>&1 |
    grep -E "Function Name|ScratchSize" | paste - - |
    grep -v "ScratchSize \[bytes/lane\]: 0 " |
    awk -v f="$(basename "$f")" '{print f, $5, $(NF-1)}'
done
rm -f /tmp/qtts_scratch_check.o
