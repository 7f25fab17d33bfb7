set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench_k1 > gpurun_out/ubench_k1_nt.log 2>&1 && bash tools/gpu_check.sh
