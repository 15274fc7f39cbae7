# final confirmation on the committed tree: GPU suite, smoke, batch 8 / 16 bench lines (C4 per-GPU shape)
#   bash tools/gpu_final.sh [tests]   (without "tests": sampler kernel tests + micro-benchmark only)
set -o pipefail
O=gpurun_out/final
mkdir -p $O
if [ "$1" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
else
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "sampler or expf" -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  timeout -k 10 60 ./tools/mb_sample > $O/mb_sample.txt 2>&1 || exit 1
  cat $O/mb_sample.txt
fi
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for b in 8 16; do
  timeout -k 10 600 python bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_b$b.json 2> $O/bench_b$b.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_b$b.json'));print('batch $b', d['value'], d['ms_per_step'])"
done
