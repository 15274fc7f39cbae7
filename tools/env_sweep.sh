#!/bin/bash
# Runtime-knob sweep of the bench (development tool).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/envsweep; mkdir -p $O; cd $R
run() { echo "== $*" >> $O/sweep.txt; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 3 > $O/tmp.json 2>> $O/sweep.err || exit 1; python3 -c "import json;d=json.load(open('$O/tmp.json'));print(d['value'], d['ms_per_step'], d['first_packet_ms'])" >> $O/sweep.txt; }
run X=1
run HIP_FORCE_DEV_KERNARG=1
run HIP_FORCE_DEV_KERNARG=0
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run AMD_DIRECT_DISPATCH=0
run ROC_SKIP_KERNEL_ARG_COPY=1
run DEBUG_HIP_GRAPH_BATCH_SIZE=64
cat $O/sweep.txt
