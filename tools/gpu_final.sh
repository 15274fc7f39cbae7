# final confirmation on the committed tree: GPU suite, smoke, batch 8 / 16 bench lines (C4 per-GPU shape)
set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for b in 8 16; do
  timeout -k 10 600 python bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_b$b.json 2> $O/bench_b$b.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_b$b.json'));print('batch $b', d['value'], d['ms_per_step'])"
done
