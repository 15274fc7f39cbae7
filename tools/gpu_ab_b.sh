# same-box A/B (lib_a vs in-tree) at batch 8 and 4, 2 rounds
set -o pipefail
bash tools/gpu_ab.sh "--batch 8 --steps 2 --warmup 1" 2 || exit 1
bash tools/gpu_ab.sh "--batch 4 --steps 2 --warmup 1" 1 || exit 1
