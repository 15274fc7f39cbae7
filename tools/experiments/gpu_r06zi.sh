#!/bin/bash
# Round 6 (r06zi, the r06w lines again on the final tree r06zf): the remaining lines -- EOS mode batch 1, voice
# clone batch 1 from reference codes and from 5 s of reference audio (first
# packet), the EOS work queue (96 utterances on 8 slots).
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06zi
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --eos --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/eos.json 2> $O/eos.err
timeout -k 10 300 python bench.py --voice-clone --vc-codes --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/vc1_codes.json 2> $O/vc1_codes.err
timeout -k 10 300 python bench.py --voice-clone --steps 3 --warmup 1 --no-cpu-baseline --no-profile > $O/vc1_audio.json 2> $O/vc1_audio.err
timeout -k 10 600 python bench.py --eos --batch 8 --queue 96 --steps 1 --warmup 0 --no-cpu-baseline --no-profile > $O/q96.json 2> $O/q96.err
for f in $O/*.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f'.split('/')[-1], d['value'], d.get('first_packet_ms'), json.dumps(d['detail'])[:200])"; done
