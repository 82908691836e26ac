#!/bin/bash
# GPU session (run on the GPU box from the repo root):
#   tools/gpu_session.sh <name> [test|bench|prof]...
# test   pytest -m gpu (one process, per-test timeout)
# bench  the driver's exact bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5)
# prof   rocprofv3 --kernel-trace --stats of that same command, plus a
#        serialised (SIFT_SERIAL=1, kernel-alone) trace; summaries via prof_summary.py
# timeline  kernel trace of synchronous detects (the latency critical path)
# apitrace  the same with the HIP runtime trace: launch call vs kernel start
# steplog   the timed region's job timeline (bench.py --step-log)
# ab/ab2/ab3  in-process interleaved A/B ($AB_ARGS ...); for anything that
#        touches streams use tools/bench_ab.sh (one process per run)
# Every GPU step has its own time limit and the steps stop at the first failure.
set -o pipefail
R=$(pwd)
N=${1:?name}
shift
O=gpurun_out/$N
mkdir -p $O
for step in "$@"; do
  case $step in
  test)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
    tail -2 $O/pytest_gpu.log ;;
  bench)
    timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
        || { tail -20 $O/bench.err; exit 1; }
    cat $O/bench.json ;;
  prof)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/$O/prof -o run \
        -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/$O/bench_prof.json 2> $R/$O/bench_prof.err \
        || { tail -20 $R/$O/bench_prof.err; exit 1; }
    SIFT_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/$O/ser -o run \
        -- python3 $R/bench.py --sync --steps 200 --warmup 10 --no-cpu-baseline --no-extra --no-matcher \
        --no-alone --no-big > $R/$O/bench_ser.json 2> $R/$O/bench_ser.err \
        || { tail -20 $R/$O/bench_ser.err; exit 1; }
    cd $R
    python tools/prof_summary.py $O/prof/run_kernel_trace.csv > $O/summary.txt
    python tools/prof_summary.py $O/ser/run_kernel_trace.csv > $O/summary_serial.txt
    cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv 2>/dev/null
    cp $O/ser/run_kernel_stats.csv $O/kernel_stats_serial.csv 2>/dev/null
    # the traces themselves are tens of MB (gpurun copies back <= 64 MiB)
    rm -rf $O/prof $O/ser
    echo PROF_DONE ;;
  ab|ab2|ab3)
    # interleaved A/B; variants and options from $AB_ARGS (resp. $AB2_ARGS, $AB3_ARGS)
    v=AB_ARGS; [ $step = ab2 ] && v=AB2_ARGS; [ $step = ab3 ] && v=AB3_ARGS
    timeout -k 10 600 python -u tools/ab_interleaved.py ${!v} > $O/$step.txt 2>&1 \
        || { tail -20 $O/$step.txt; exit 1; }
    grep -v amdgpu.ids $O/$step.txt ;;
  timeline)
    # kernels of synchronous detects on their real streams (start / end /
    # queue per dispatch of one image): the latency critical path
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/lat -o run \
        -- python3 $R/bench.py --sync --steps 100 --warmup 10 --no-cpu-baseline --no-extra \
        --no-matcher --no-alone --no-big --no-events > $R/$O/bench_lat.json 2> $R/$O/bench_lat.err \
        || { tail -20 $R/$O/bench_lat.err; exit 1; }
    cd $R
    python tools/prof_summary.py $O/lat/run_kernel_trace.csv > $O/summary_lat.txt
    rm -rf $O/lat
    tail -45 $O/summary_lat.txt ;;
  apitrace)
    # host enqueue vs device execution of synchronous detects (HIP runtime
    # trace joined with the kernel trace, tools/prof_api.py)
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace \
        --output-format csv -d $R/$O/api -o run \
        -- python3 $R/bench.py --sync --steps 30 --warmup 5 --no-cpu-baseline --no-extra \
        --no-matcher --no-alone --no-big --no-events > $R/$O/bench_api.json 2> $R/$O/bench_api.err \
        || { tail -20 $R/$O/bench_api.err; exit 1; }
    cd $R
    python tools/prof_api.py $O/api > $O/api.txt 2>&1
    rm -rf $O/api
    head -80 $O/api.txt ;;
  steplog)
    # the driver's bench shape with the timed region's submit / fetch / done times
    timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-matcher \
        --no-alone --no-big --no-extra --step-log > $O/steplog.json 2> $O/steplog.err \
        || { tail -20 $O/steplog.err; exit 1; }
    grep -A70 "step log" $O/steplog.err ;;
  big)
    # BASELINE configs 3 and 5: job timeline with host phases (untraced),
    # rocprofv3 kernel trace of the pipelined leg (2 jobs in flight) and of
    # a serialised context (kernels alone); $BIG_CONFIGS, $BIG_IMAGES
    for cfg in ${BIG_CONFIGS:-config3 config5}; do
      timeout -k 10 300 python3 tools/big_profile.py $cfg --images ${BIG_IMAGES:-12} \
          > $O/big_$cfg.json 2> $O/big_$cfg.err || { tail -20 $O/big_$cfg.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/big_$cfg.json')); print('$cfg', d['ms_per_image'], d['keypoints_per_image'])"
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/$O/b_$cfg -o run \
          -- python3 $R/tools/big_profile.py $cfg --images ${BIG_IMAGES:-12} \
          > $R/$O/big_prof_$cfg.json 2> $R/$O/big_prof_$cfg.err \
          || { tail -20 $R/$O/big_prof_$cfg.err; exit 1; }
      SIFT_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/$O/bs_$cfg -o run \
          -- python3 $R/tools/big_profile.py $cfg --images 4 --sync \
          > $R/$O/big_ser_$cfg.json 2> $R/$O/big_ser_$cfg.err \
          || { tail -20 $R/$O/big_ser_$cfg.err; exit 1; }
      cd $R
      python tools/prof_summary.py $O/b_$cfg/run_kernel_trace.csv > $O/summary_$cfg.txt
      python tools/prof_summary.py $O/bs_$cfg/run_kernel_trace.csv > $O/summary_serial_$cfg.txt
      python tools/prof_timeline.py $O/b_$cfg/run_kernel_trace.csv > $O/timeline_$cfg.txt
      rm -rf $O/b_$cfg $O/bs_$cfg
    done
    echo BIG_DONE ;;
  bigdepth)
    # the BASELINE config 3 / 5 legs at 2 and 3 jobs in flight (bench.py legs only)
    for d in 2 3; do
      SIFT_BIG_DEPTH=$d timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-extra \
          --no-alone --no-cpu-baseline --no-matcher > $O/bigdepth_$d.json 2> $O/bigdepth_$d.err \
          || { tail -20 $O/bigdepth_$d.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/bigdepth_$d.json')); print('depth $d', [(c, round(d[c]['ms_per_image'],3), d[c]['host_phases_ms']) for c in ('config3','config5')])"
    done ;;
  divcheck)
    timeout -k 10 300 tools/divcheck > $O/divcheck.txt 2>&1 || { tail -5 $O/divcheck.txt; exit 1; }
    tail -3 $O/divcheck.txt ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo SESSION_DONE
