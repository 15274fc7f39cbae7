#!/bin/bash
# Round-5 pass ad: refresh the EOS-mode line and the voice-clone batch-1 line
# (first packet from reference codes and from reference audio) on the final tree
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05ad
mkdir -p $O
cd $R
timeout -k 10 600 python bench.py --eos --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/bench_eos.json 2> $O/bench_eos.err
python -c "import json; d=json.loads(open('$O/bench_eos.json').read().strip().splitlines()[-1]); print('eos', d['value'], d.get('eos_mode'), d.get('first_packet_ms'))"
timeout -k 10 600 python bench.py --voice-clone --no-cpu-baseline --no-profile --steps 3 --warmup 1 > $O/bench_vc1.json 2> $O/bench_vc1.err
python -c "import json; d=json.loads(open('$O/bench_vc1.json').read().strip().splitlines()[-1]); print('vc1', d['value'], d.get('detail'))"
