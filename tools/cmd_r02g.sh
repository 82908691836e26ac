set -o pipefail
SIFT_SERIAL=1 tools/gpu_prof.sh r02g_serial "--steps 60 --warmup 5 --sync" || exit 1
tools/gpu_prof.sh r02g_b8 "--steps 40 --warmup 5 --batch 8" || exit 1
