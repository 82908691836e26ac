set -o pipefail
bash tools/pmc_kp.sh r02ar/sq > gpurun_out/r02ar_sq.log 2>&1 || { tail gpurun_out/r02ar_sq.log; exit 1; }
echo done
