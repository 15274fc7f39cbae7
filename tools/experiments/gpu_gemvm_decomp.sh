set -o pipefail
cd /tmp && export TMPDIR=/tmp
VARIANTS=${VARIANTS:-0 1 2 3}
SHAPES=${SHAPES:-talker_qkv talker_o talker_gate_up talker_down st_qkv st_gate_up st_down}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/dec
for s in $SHAPES; do
  for v in $VARIANTS; do
    QTTS_GM_DBG=$v timeout -k 10 90 rocprofv3 --kernel-trace -f csv -d /tmp/dec_${s}_$v -o run -- python3 $R/tools/mb_gemvm.py --only $s --batch 8 --n 100 > /dev/null 2>&1 || exit 1
    f=$(ls /tmp/dec_${s}_$v/*/run_kernel_trace.csv 2>/dev/null | head -1)
    [ -n "$f" ] || f=$(find /tmp/dec_${s}_$v -name "*kernel_trace.csv" | head -1)
    echo "$s dbg=$v $(python3 $R/tools/trace_by_grid.py $f 3 | grep k_gemvm | head -1)"
  done
done
