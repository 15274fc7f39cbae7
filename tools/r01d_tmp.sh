set -eo pipefail
O=gpurun_out/r01as; mkdir -p $O
timeout -k 10 300 python3 tools/prof_stream.py > $O/stream.txt 2>&1
QTTS_HIP_CODEC_G1=0 timeout -k 10 300 python3 tools/prof_stream.py > $O/stream_off.txt 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 > $O/b1.json 2> $O/b1.err
QTTS_HIP_CODEC_G1=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 > $O/b0.json 2> $O/b0.err
echo done
