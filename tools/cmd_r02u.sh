set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02u
mkdir -p $O
timeout -k 10 300 python -u tools/ab_interleaved.py --rounds 6 --steps 400 base SIFT_EXT_WAVES=3072 SIFT_EXT_WAVES=6144 SIFT_EXT_WAVES=12288 SIFT_REFINE_WGS=128 SIFT_KP_WGS=384 2>&1 | tee $O/ab1.txt || exit 1
cd /tmp && export TMPDIR=/tmp
for v in 4096 6144 12288; do
SIFT_EXT_WAVES=$v SIFT_REFINE_WGS=128 SIFT_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/ser$v -o run -- python3 $R/bench.py --sync --steps 100 --warmup 10 --no-cpu-baseline --no-extra --no-matcher --no-events > $O/ser$v.json 2> $O/ser$v.err || { tail -5 $O/ser$v.err; exit 1; }
echo "waves $v"; grep -E "extrema|refine" $O/ser$v/run_kernel_stats.csv | cut -d, -f1-5
done
cd $R && bash tools/pmc_kp.sh r02u/sq > $O/sq.log 2>&1 || { tail $O/sq.log; exit 1; }
