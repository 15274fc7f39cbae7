set -eo pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r01ad; mkdir -p $O; rm -f gpurun_out/envsweep/sweep.txt
timeout -k 10 900 bash tools/env_sweep.sh "X=1" "QTTS_HIP_CONV_SPLIT=0" "X=2" > $O/sweep_out.txt 2>&1
cp gpurun_out/envsweep/tmp.json $O/last_bench.json
echo done
