set -eo pipefail
O=gpurun_out/r01aq; mkdir -p $O; rm -f gpurun_out/envsweep/sweep.txt
timeout -k 10 1000 bash tools/env_sweep.sh "X=1" "QTTS_HIP_XADD_TARGET=256" "QTTS_HIP_XADD_TARGET=128" "QTTS_HIP_XADD_TARGET=1024" "X=2" > $O/sweep_out.txt 2>&1
echo done
