# batch split-K on / off (QTTS_HIP_BSPLIT=0), same box, alternating
set -o pipefail
mkdir -p gpurun_out/bs
for i in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export QTTS_HIP_BSPLIT=0; else unset QTTS_HIP_BSPLIT; fi
    for b in 8 4; do
      timeout -k 10 300 python3 bench.py --batch $b --steps 2 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/bs/$v.json 2> gpurun_out/bs/$v.err || exit 1
      python3 -c "import json;d=json.load(open('gpurun_out/bs/$v.json'));print('$v batch $b', d['value'], d['ms_per_step'])"
    done
  done
done
