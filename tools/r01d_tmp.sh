set -eo pipefail
O=gpurun_out/r01i; mkdir -p $O; rm -f gpurun_out/envsweep/sweep.txt
timeout -k 10 900 bash tools/env_sweep.sh "X=1" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "AMD_DIRECT_DISPATCH=0" "DEBUG_HIP_GRAPH_BATCH_SIZE=64" "GPU_STREAMOPS_CP_WAIT=1" > $O/sweep_out.txt 2>&1
echo done
