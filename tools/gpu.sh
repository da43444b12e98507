#!/bin/bash
# The one GPU-box runner: tools/gpu.sh TAG STEP [STEP ...]
#
# Runs the named steps in order on the box, every GPU step under its own time
# limit; the first step that fails (a test failure excepted) ends the script,
# so nothing more touches the GPU after a crash, abort or timeout.  Results go
# to gpurun_out/*_TAG.*; copy the ones worth keeping into profiles/rN/.
#
# Steps:
#   build          make clean + hipcc gfx950 build of libtmhip (and libtmh5
#                  when libhdf5 is there) from the pushed sources, toolchain
#                  and sha256 logged (build_TAG.log)
#   tests          pytest -m gpu, then smoke (gpu_tests_TAG.log, smoke_TAG.log)
#   bench          the default bench line, CPU baseline included (bench_TAG.json)
#   quick          bench --steps 10 --no-extras --cpu-sample 0 (bench_quick_TAG.json)
#   bright         quick on bright data (bench_bright_TAG.json)
#   repeat:N       N more quick bench processes (bench_repeat_TAG.jsonl)
#   dist432        one rank, forced-distributed, 4 channels x 432 sites: each
#                  GPU's share of configs[2] at N = 8 (dist432_TAG.json)
#   pytest:EXPR    the GPU tests selected by -k EXPR, '+' for spaces (gpu_tests_k_TAG.log)
#   input[:N]      tools/bench_input.py on N full-size gzip files (host and GPU
#                  decode, run_job, the sharded job) -> bench_input_TAG.json
#   dist432v:ARGS  dist432 with extra flags ('+' for spaces) -> dist432_v_TAG.jsonl
#   prof432        rocprofv3 kernel trace of dist432 -> rocprof_dist432_TAG/
#   prof:DIST      rocprofv3 --kernel-trace --stats of a short bench on DIST
#                  (synthetic | bright) -> rocprof_DIST_TAG/
#   profh[:DIST]   prof with the HIP runtime trace (host waits) -> rocprof_h_DIST_TAG/
#   pmc:DIST       FETCH_SIZE and WRITE_SIZE passes (each its own run) of a
#                  short bench on DIST -> pmc_traffic_DIST_TAG.json
#   ab:R:LIB,LIB   same-box A/B of library builds (TMH_LIB), R rounds, the
#                  order reversed every other round (ab_TAG.jsonl)
#   ab432:R:LIB,.. the same over dist432 runs (ab432_TAG.jsonl)
# BENCH_ARGS adds flags to every bench run of quick/bright/repeat/ab/prof/pmc.
set -u
TAG=$1
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
QB="bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-extras ${BENCH_ARGS:-}"
# (the profiled bench keeps its own event timing: its line and the rocprof
# summary then describe the same process)
SB="bench.py --steps 5 --warmup 2 --cpu-sample 0 --no-extras ${BENCH_ARGS:-}"

summ() {  # one-line summary of a bench JSON line
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.strip()][-1]); r=d.get('roofline') or {}; print(sys.argv[1], d['value'], d['ms_per_step'], d.get('check_vs_oracle'), r.get('frac'), {k: v['avg_ms'] for k, v in d.get('kernels', {}).items()})" "$1"
}

for step in "$@"; do
  IFS=: read -r name a1 a2 <<< "$step"
  echo "== $step"
  case $name in
    build)
      L=$O/build_$TAG.log
      { /opt/rocm/bin/hipcc --version; echo; } > $L 2>&1
      timeout -k 10 120 make -C tmlibrary_amd/csrc clean >> $L 2>&1 || exit $?
      timeout -k 10 900 make -C tmlibrary_amd/csrc -j16 >> $L 2>&1 || exit $?
      if [ -f /opt/conda/include/hdf5.h ]; then
        timeout -k 10 300 make -C tmlibrary_amd/csrc h5 >> $L 2>&1 || exit $?
      fi
      sha256sum tmlibrary_amd/hip/*.so | tee -a $L
      ;;
    tests)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -v -ra --timeout 300 --timeout-method thread > $O/gpu_tests_$TAG.log 2>&1
      rc=$?
      echo "pytest rc=$rc" >> $O/gpu_tests_$TAG.log
      grep -E "passed|failed" $O/gpu_tests_$TAG.log | tail -3
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
      timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke_$TAG.log 2>&1 || exit $?
      tail -2 $O/smoke_$TAG.log
      if [ $rc -ne 0 ]; then exit $rc; fi
      ;;
    bench)
      timeout -k 10 900 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || exit $?
      summ $O/bench_$TAG.json
      ;;
    quick)
      timeout -k 10 300 python $QB > $O/bench_quick_$TAG.json 2> $O/bench_quick_$TAG.err || exit $?
      summ $O/bench_quick_$TAG.json
      ;;
    bright)
      timeout -k 10 300 python $QB --distribution bright > $O/bench_bright_$TAG.json 2> $O/bench_bright_$TAG.err || exit $?
      summ $O/bench_bright_$TAG.json
      ;;
    repeat)
      : > $O/bench_repeat_$TAG.jsonl
      for i in $(seq 1 ${a1:-5}); do
        timeout -k 10 300 python $QB > $O/b.tmp 2>> $O/bench_repeat_$TAG.err || exit $?
        cat $O/b.tmp >> $O/bench_repeat_$TAG.jsonl
        summ $O/b.tmp
      done
      ;;
    dist432)
      TMH_BENCH_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 \
        timeout -k 10 300 python bench.py --layout sharded --channels 4 --sites 432 --steps 10 \
        --warmup 3 --no-extras --cpu-sample 0 ${BENCH_ARGS:-} > $O/dist432_$TAG.json 2> $O/dist432_$TAG.err || exit $?
      summ $O/dist432_$TAG.json
      ;;
    dist432v)
      # one variant: dist432v:--flag+value+--flag2 ('+' for spaces), appended to dist432_v_TAG.jsonl
      V=$(echo "$a1" | tr '+' ' ')
      TMH_BENCH_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 \
        timeout -k 10 300 python bench.py --layout sharded --channels 4 --sites 432 --steps 10 \
        --warmup 3 --no-extras --cpu-sample 0 ${BENCH_ARGS:-} $V > $O/dist432v.tmp 2>> $O/dist432_v_$TAG.err || exit $?
      python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.strip()][-1]); print(json.dumps({'variant': sys.argv[2], 'value': d['value'], 'ms': d['ms_per_step'], 'host_ms': d.get('host_queue_ms_per_step'), 'check': d['check_vs_oracle'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" $O/dist432v.tmp "$V" | tee -a $O/dist432_v_$TAG.jsonl
      ;;
    ab432)
      # dist432 A/B over libraries: ab432:ROUNDS:LIB1,LIB2 (LIB may carry '+'-joined flags)
      IFS=, read -r -a LIBS <<< "$a2"
      : > $O/ab432_$TAG.jsonl
      for i in $(seq 1 ${a1:-3}); do
        ORDER=("${LIBS[@]}")
        if [ $((i % 2)) -eq 0 ]; then
          ORDER=(); for ((j=${#LIBS[@]}-1; j>=0; j--)); do ORDER+=("${LIBS[j]}"); done
        fi
        for L in "${ORDER[@]}"; do
          IFS=+ read -r -a LA <<< "$L"
          TMH_LIB=${LA[0]} TMH_BENCH_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 \
            MASTER_PORT=29517 timeout -k 10 300 python bench.py --layout sharded --channels 4 --sites 432 \
            --steps 10 --warmup 3 --no-extras --cpu-sample 0 "${LA[@]:1}" > $O/ab432_$TAG.tmp 2>> $O/ab432_$TAG.err || exit $?
          python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[2]) if l.strip()][-1]); print(json.dumps({'lib': sys.argv[1], 'value': d['value'], 'ms': d['ms_per_step'], 'check': d['check_vs_oracle'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" "$L" $O/ab432_$TAG.tmp >> $O/ab432_$TAG.jsonl
          tail -1 $O/ab432_$TAG.jsonl
        done
      done
      ;;
    prof432)
      TMH_BENCH_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 \
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rocprof_dist432_$TAG -o run \
        -- python3 bench.py --layout sharded --channels 4 --sites 432 --steps 5 --warmup 2 \
        --no-extras --cpu-sample 0 ${BENCH_ARGS:-} > $O/rocprof_dist432_$TAG.json 2> $O/rocprof_dist432_$TAG.log || exit $?
      summ $O/rocprof_dist432_$TAG.json
      ;;
    prof432h)
      # prof432 with the HIP runtime calls (host waits) on the kernels' clock:
      # prof432h[:ARGS] ('+' for spaces) -> rocprof_dist432h_TAG/
      V=$(echo "${a1:-}" | tr '+' ' ')
      TMH_BENCH_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 \
        timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace \
        --output-format csv -d $O/rocprof_dist432h_$TAG -o run \
        -- python3 bench.py --layout sharded --channels 4 --sites 432 --steps 5 --warmup 2 \
        --no-extras --cpu-sample 0 ${BENCH_ARGS:-} $V > $O/rocprof_dist432h_$TAG.json 2> $O/rocprof_dist432h_$TAG.log || exit $?
      summ $O/rocprof_dist432h_$TAG.json
      ;;
    input)
      timeout -k 10 600 python tools/bench_input.py --sites ${a1:-256} --threads 16 --repeat 4 \
        > $O/bench_input_$TAG.json 2> $O/bench_input_$TAG.err || exit $?
      tail -c 1500 $O/bench_input_$TAG.json
      ;;
    inflate)
      # GPU inflate kernels -> bench_inflate_TAG.json
      timeout -k 10 600 python tools/bench_inflate.py --block 128 \
        > $O/bench_inflate_$TAG.json 2> $O/bench_inflate_$TAG.err || exit $?
      tail -c 600 $O/bench_inflate_$TAG.json
      ;;
    pytest)
      # a subset of the GPU tests: pytest:EXPR (-k expression, '+' for spaces)
      K=$(echo "$a1" | tr '+' ' ')
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -ra --timeout 300 --timeout-method thread \
        -k "$K" > $O/gpu_tests_k_$TAG.log 2>&1
      rc=$?
      grep -E "passed|failed" $O/gpu_tests_k_$TAG.log | tail -3
      if [ $rc -ne 0 ]; then exit $rc; fi
      ;;
    prof)
      D=${a1:-synthetic}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rocprof_${D}_$TAG -o run \
        -- python3 $SB --distribution $D > $O/rocprof_${D}_$TAG.json 2> $O/rocprof_${D}_$TAG.log || exit $?
      summ $O/rocprof_${D}_$TAG.json
      ;;
    profh)
      # prof with the HIP runtime calls on the kernels' clock: profh[:DIST]
      D=${a1:-synthetic}
      timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace \
        --output-format csv -d $O/rocprof_h_${D}_$TAG -o run \
        -- python3 $SB --distribution $D > $O/rocprof_h_${D}_$TAG.json 2> $O/rocprof_h_${D}_$TAG.log || exit $?
      summ $O/rocprof_h_${D}_$TAG.json
      ;;
    pmc)
      D=${a1:-synthetic}
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${c}_${D}_$TAG -o run \
          -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-extras --no-profile --distribution $D \
          > $O/pmc_${c}_${D}_$TAG.log 2>&1 || exit $?
      done
      python3 tools/pmc_traffic.py $O/pmc_FETCH_SIZE_${D}_$TAG $O/pmc_WRITE_SIZE_${D}_$TAG --sites 3456 \
        --height 2160 --width 2560 --distribution $D -o $O/pmc_traffic_${D}_$TAG.json || exit $?
      ;;
    pmcinstall)
      # the pmc:DIST result of this call as the bench's traffic file (so a
      # bench later in the same call reports roofline.traffic for this build)
      D=${a1:-synthetic}
      SUF=""; [ "$D" != "synthetic" ] && SUF="_$D"
      cp $O/pmc_traffic_${D}_$TAG.json profiles/pmc_traffic${SUF}.json || exit $?
      mkdir -p $O/profiles && cp $O/pmc_traffic_${D}_$TAG.json $O/profiles/pmc_traffic${SUF}.json
      ;;
    avail)
      timeout -k 10 60 rocprofv3 --list-avail > $O/pmc_avail_$TAG.txt 2>&1 || exit $?
      grep -cE "SQ_|GRBM_" $O/pmc_avail_$TAG.txt || true
      ;;
    pmcsq)
      # SQ / GRBM counters of a short bench on DIST, two passes (each <= 8 SQ
      # and <= 2 GRBM counters, its own run): pmcsq[:DIST] -> pmc_sq_DIST_TAG.json
      D=${a1:-synthetic}
      PA="SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
      PB="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
      n=0
      for P in "$PA" "$PB"; do
        n=$((n + 1))
        timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $O/pmcsq${n}_${D}_$TAG -o run \
          -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-extras --no-profile --no-box \
          --jobs-in-flight 1 --distribution $D > $O/pmcsq${n}_${D}_$TAG.log 2>&1 || exit $?
      done
      python3 tools/pmc_sq.py $O/pmcsq1_${D}_$TAG $O/pmcsq2_${D}_$TAG --pixels $((3456 * 2160 * 2560)) \
        -o $O/pmc_sq_${D}_$TAG.json > /dev/null || exit $?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(k[:60], v['derived']) for k, v in d['kernels'].items()]" $O/pmc_sq_${D}_$TAG.json
      ;;
    ab)
      IFS=, read -r -a LIBS <<< "$a2"
      : > $O/ab_$TAG.jsonl
      for i in $(seq 1 ${a1:-3}); do
        ORDER=("${LIBS[@]}")
        if [ $((i % 2)) -eq 0 ]; then
          ORDER=(); for ((j=${#LIBS[@]}-1; j>=0; j--)); do ORDER+=("${LIBS[j]}"); done
        fi
        for L in "${ORDER[@]}"; do
          # LIB may carry bench flags after a '+': path+--fused-config+3
          IFS=+ read -r -a LA <<< "$L"
          TMH_LIB=${LA[0]} timeout -k 10 300 python $QB "${LA[@]:1}" > $O/ab_$TAG.tmp 2>> $O/ab_$TAG.err || exit $?
          python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[2]) if l.strip()][-1]); print(json.dumps({'lib': sys.argv[1], 'value': d['value'], 'ms': d['ms_per_step'], 'check': d['check_vs_oracle'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" "$L" $O/ab_$TAG.tmp >> $O/ab_$TAG.jsonl
          tail -1 $O/ab_$TAG.jsonl
        done
      done
      ;;
    mb)
      # a microbenchmark built here: mb:NAME[:ARGS] ('+' for spaces) -> mb_NAME_TAG.txt
      V=$(echo "${a2:-}" | tr '+' ' ')
      timeout -k 10 180 ./tools/mb/$a1 $V > $O/mb_${a1}_$TAG.txt 2>&1 || { tail -5 $O/mb_${a1}_$TAG.txt; exit 1; }
      tail -20 $O/mb_${a1}_$TAG.txt
      ;;
    abenv|abenvb|abenv432)
      # A/B over environment settings of one library: abenv:R:VAR=a,VAR=b (each
      # entry may join several VAR=value with '+'), order reversed every other
      # round; abenv = quick bench, abenvb = quick bench on bright data,
      # abenv432 = the dist432 run
      IFS=, read -r -a ENVS <<< "$a2"
      : > $O/${name}_$TAG.jsonl
      case $name in
        abenv) CMD="python $QB"; DE="" ;;
        abenvb) CMD="python $QB --distribution bright"; DE="" ;;
        abenv432) CMD="python bench.py --layout sharded --channels 4 --sites 432 --steps 10 --warmup 3 --no-extras --cpu-sample 0 ${BENCH_ARGS:-}"
          DE="TMH_BENCH_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517" ;;
      esac
      for i in $(seq 1 ${a1:-3}); do
        ORDER=("${ENVS[@]}")
        if [ $((i % 2)) -eq 0 ]; then
          ORDER=(); for ((j=${#ENVS[@]}-1; j>=0; j--)); do ORDER+=("${ENVS[j]}"); done
        fi
        for E in "${ORDER[@]}"; do
          EV=$(echo "$E" | tr '+' ' ')
          env $EV $DE timeout -k 10 300 $CMD > $O/${name}_$TAG.tmp 2>> $O/${name}_$TAG.err || exit $?
          python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[2]) if l.strip()][-1]); print(json.dumps({'env': sys.argv[1], 'value': d['value'], 'ms': d['ms_per_step'], 'check': d['check_vs_oracle'], 'k': {k: v['avg_ms'] for k, v in d['kernels'].items()}}))" "$E" $O/${name}_$TAG.tmp >> $O/${name}_$TAG.jsonl
          tail -1 $O/${name}_$TAG.jsonl
        done
      done
      ;;
    *)
      echo "unknown step $step"; exit 2
      ;;
  esac
done
echo "$TAG-ok"
