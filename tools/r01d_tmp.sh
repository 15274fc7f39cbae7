set -eo pipefail
O=gpurun_out/r01o; mkdir -p $O; rm -f gpurun_out/envsweep/sweep.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -k "conv or codec or e2e or full or stream" -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 python3 tools/prof_codec.py > $O/codec_run.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/codec -o run -- python3 tools/prof_codec.py > $O/codec_prof.log 2>&1
python3 tools/prof_codec.py --summarize $O/codec > $O/codec_summary.txt
timeout -k 10 900 bash tools/env_sweep.sh "X=1" "QTTS_HIP_CONV_TILES=32" "QTTS_HIP_CONV_TILES=48" > $O/sweep_out.txt 2>&1
echo done
