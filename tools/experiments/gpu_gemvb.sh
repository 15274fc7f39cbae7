# k_gemvb (x sliced per wave) vs k_gemvm (x staged per workgroup): the GPU
# suite on the default (k_gemvb) build, isolated batch GEMV shapes under
# rocprofv3 for both (QTTS_HIP_GEMVB=0 selects k_gemvm), then same-box
# bench.py batch-8 / 16 lines alternating the two.
#   bash tools/gpu_gemvb.sh <tag> [tests|notests]
set -o pipefail
TAG=${1:-gb}
MODE=${2:-tests}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ "$MODE" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
fi
export TMPDIR=/tmp
for g in 1 0; do
  rm -rf /tmp/gs$g
  QTTS_HIP_GEMVB=$g timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d /tmp/gs$g -o run -- python3 $GRAFT_REPO_ROOT/tools/mb_gemvm.py --batch 8 --n 100 > $O/mb_g$g.log 2>&1 || exit 1
  f=$(find /tmp/gs$g -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_by_grid.py $f 20 > $O/shapes_b8_gemvb$g.txt
  cat $O/shapes_b8_gemvb$g.txt
done
for b in 8 16; do
  for r in 1 2; do
    for g in 1 0; do
      QTTS_HIP_GEMVB=$g timeout -k 10 400 python3 bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/bench_b${b}_g${g}_r$r.json 2> $O/bench_b${b}_g${g}_r$r.err || exit 1
      python3 -c "import json;d=json.load(open('$O/bench_b${b}_g${g}_r$r.json'));print('batch $b gemvb=$g', d['value'], d['ms_per_step'])"
    done
  done
done
