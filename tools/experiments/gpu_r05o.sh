#!/bin/bash
# Round-5 pass o: where a 128-frame codec decode's time goes (current build)
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05o
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/prof_codec.py > $O/plain.txt 2>&1
cat $O/plain.txt | grep decode
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/codec -o run -- python3 tools/prof_codec.py > $O/prof.log 2>&1
python3 tools/prof_codec.py --summarize $O/codec > $O/codec_kernels.txt
head -45 $O/codec_kernels.txt
