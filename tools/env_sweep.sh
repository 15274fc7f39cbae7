#!/bin/bash
# Runtime-knob sweep of the bench (development tool).  Each argument is one
# case: a space-separated list of VAR=value settings ("X=1" = defaults).
#   bash tools/env_sweep.sh "X=1" "QTTS_HIP_ATT_PRO=0" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/envsweep; mkdir -p $O; cd $R
run() {
  echo "== $*" >> $O/sweep.txt
  env $* timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 > $O/tmp.json 2>> $O/sweep.err || exit 1
  python3 -c "
import json; d = json.load(open('$O/tmp.json')); fp = d.get('frame_profile', {})
print(d['value'], d['ms_per_step'], d['first_packet_ms'], fp.get('kernel_ms_per_frame'), fp.get('n_kernels'))
for k, v in list(fp.get('kernels', {}).items())[:6]: print('   ', k, v)" >> $O/sweep.txt
}
for c in "$@"; do run $c; done
cat $O/sweep.txt
