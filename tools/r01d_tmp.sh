set -eo pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r01ax7; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "conv or codec or snake" > $O/conv_tests.log 2>&1
for e in X=1 QTTS_HIP_CONV_WN=2; do echo "== $e" >> $O/codec_times.txt; env $e timeout -k 10 120 python3 tools/prof_codec.py >> $O/codec_times.txt 2>&1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/codec -o run -- python3 $R/tools/prof_codec.py > $O/run.log 2>&1
python3 $R/tools/prof_codec.py --summarize $O/codec > $O/summary.txt 2>&1
rm -rf $O/codec
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 3 > $O/bench1.json 2> $O/err.txt
echo done
