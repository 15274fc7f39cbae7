set -eo pipefail
O=gpurun_out/r01am; mkdir -p $O; rm -f gpurun_out/envsweep/sweep.txt
timeout -k 10 1000 bash tools/env_sweep.sh "X=1" "QTTS_HIP_PF_WG=224" "QTTS_HIP_PF_WG=224 QTTS_HIP_PF_GU=0" "QTTS_HIP_PF_WG=224 QTTS_HIP_PF_GU=12" "QTTS_HIP_PF_WG=112 QTTS_HIP_PF_GU=12" > $O/sweep_out.txt 2>&1
echo done
