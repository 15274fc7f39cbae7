#!/bin/bash
# Round-5 first pass: the XCD premise of the L2 prefetch, EOS stop steps for
# the EOS golden, the bench line with the measured stream bandwidth, and the
# keep/drop A/B of the L2 prefetch with 4 alternating processes per arm.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05a
mkdir -p $O
cd $R
timeout -k 10 90 ./tools/mb_l2pf > $O/mb_l2pf.txt 2>&1
cat $O/mb_l2pf.txt
timeout -k 10 400 python tools/eos_stop_probe.py 1234 1235 1236 1237 1238 1239 > $O/eos_probe.txt 2> $O/eos_probe.err
cat $O/eos_probe.txt
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
python - $O/bench.json <<'PY'
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["roofline"]["achieved"], d["roofline"].get("measured_stream"))
PY
for i in 1 2 3 4; do
  QTTS_HIP_L2PF=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 10 --warmup 2 > $O/ab_off_$i.json 2> $O/ab_off_$i.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 10 --warmup 2 > $O/ab_on_$i.json 2> $O/ab_on_$i.err
  python -c "import json; f=lambda p: json.loads(open(p).read().strip().splitlines()[-1])['value']; print('pair $i off', f('$O/ab_off_$i.json'), 'on', f('$O/ab_on_$i.json'))"
done
# batch-8 sub-talker stamps (pass 5, layer 2) from the stamp build
QTTS_LIB=$R/qwen3-tts-c_amd/lib_s/libqwen_tts_amd.so QTTS_HIP_GM_DBG=99 timeout -k 10 300 python bench.py --batch 8 --steps 1 --warmup 0 --no-profile --no-cpu-baseline > $O/st_b8.json 2> $O/st_b8.err
grep gm_dbg $O/st_b8.err | tail -20
QTTS_LIB=$R/qwen3-tts-c_amd/lib_s/libqwen_tts_amd.so QTTS_HIP_GM_DBG=99 timeout -k 10 300 python bench.py --batch 1 --steps 1 --warmup 0 --no-profile --no-cpu-baseline > $O/st_b1.json 2> $O/st_b1.err
grep gm_dbg $O/st_b1.err | tail -20
echo done
