set -eo pipefail
O=gpurun_out/r01aw; mkdir -p $O; rm -f $O/configs.txt
for e in "X=1" "QWEN_TTS_HIP_OVERLAP=1" "QWEN_TTS_HIP_OVERLAP=1 QTTS_HIP_CODEC_CUS=32" "QWEN_TTS_HIP_OVERLAP=1 QTTS_HIP_CODEC_CUS=32 QTTS_HIP_CU_MASK_STYLE=1" "QWEN_TTS_HIP_OVERLAP=1 QTTS_HIP_CODEC_CUS=64 QTTS_HIP_CU_MASK_STYLE=1" "QWEN_TTS_HIP_OVERLAP=1 QTTS_HIP_CODEC_CUS=16 QTTS_HIP_CU_MASK_STYLE=1" "QTTS_HIP_CODEC_CUS=32 QTTS_HIP_CU_MASK_STYLE=1"; do
  echo "== $e" >> $O/configs.txt
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 3 > $O/tmp.json 2>> $O/err.txt
  python3 -c "
import json; d = json.load(open('$O/tmp.json'))
print(d['value'], d['ms_per_step'], d.get('first_packet_ms'))" >> $O/configs.txt
done
echo done
