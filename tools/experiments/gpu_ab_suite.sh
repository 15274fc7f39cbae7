# Same-box A/B of two builds: the GPU suite on the in-tree build, then
# bench.py alternating lib_a (QTTS_LIB) and the in-tree lib.
#   bash tools/gpu_ab_suite.sh <tag> [tests|notests] [batch sizes, default "1 8"]
set -o pipefail
TAG=${1:-ab}
MODE=${2:-tests}
BATCHES=${3:-"1 8"}
O=gpurun_out/$TAG
mkdir -p $O
if [ "$MODE" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
for b in $BATCHES; do
  rounds=1; [ $b = 1 ] && rounds=2
  bash tools/gpu_ab.sh "--batch $b --steps 3 --warmup 1" $rounds > $O/ab_b$b.txt 2>&1 || exit 1
  cat $O/ab_b$b.txt
done
