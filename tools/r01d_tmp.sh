set -eo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r01ab; mkdir -p $O; rm -f gpurun_out/envsweep/sweep.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -k "codec or stream or e2e or full or conv" -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 python3 tools/prof_stream.py > $O/stream.txt 2>&1
QTTS_HIP_CONV_SPLIT=0 timeout -k 10 300 python3 tools/prof_stream.py > $O/stream_off.txt 2>&1
timeout -k 10 300 python3 tools/prof_codec.py > $O/codec_run.log 2>&1
QTTS_HIP_CONV_SPLIT=0 timeout -k 10 300 python3 tools/prof_codec.py > $O/codec_run_off.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/streamprof -o run -- python3 $GRAFT_REPO_ROOT/tools/prof_stream.py > $O/stream_prof.txt 2>&1
echo done
