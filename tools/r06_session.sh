#!/bin/bash
# Round 6 GPU sessions: per-rank launches of an N-GPU cfg3 run (--local-banks),
# kernel stats and PMC passes (one counter group per run, MI355X_MICROARCH.md
# §rocprofv3), SQ counters beside the pure-read probe, tests, bench.
#   usage: tools/r06_session.sh TAG [steps...]
#   steps: smoke tests tests_K[+K2...] bench bench_CFG list ab_SUITE[:v1,v2,...]
#          prof_CFG[_lbN] pmc_CFG[_lbN] sq_CFG[_lbN] cold_CFG typed typedprof typedpmc typedsq
#          ab_SUITE getband getbandz ceil_kurt kurtprof_CFG kurtpmc_CFG kurtsweep
#          gloo_N_CFG hostbound typedw_N benchpipe_CFG cold_CFG[_kSTEPS]
# CFG[_lbN]: a config, optionally with --local-banks N (one rank's launch of an
# (8/N)-GPU run).  Every GPU step has its own time limit; after any failure
# nothing more runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06a}; shift || true
STEPS=${*:-"smoke tests"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "== $name failed (rc=$rc): stopping GPU work"; exit $rc; fi
}

bench_args() {  # CFG[_lbN] -> bench.py arguments for a short profiled run
  local c=${1%%_lb*} lb=""
  [ "$c" != "$1" ] && lb="--local-banks ${1##*_lb}"
  echo "--config $c $lb --steps 20 --warmup 5 --no-cpu-baseline"
}

SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"

for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as e; e.smoke()" ;;
    list) run list 120 rocprofv3 -L ;;
    tests) run tests 1100 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
          --timeout-method thread ;;
    tests_*) K=${s#tests_}  # tests_a+b: -k "a or b"
      run "$s" 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
          --timeout-method thread -k "${K//+/ or }" ;;
    bench) run bench 600 python bench.py ;;
    benchpipe_*) run "$s" 600 python bench.py --config "${s#benchpipe_}" --pipeline --no-cpu-baseline ;;
    bench_*) run "$s" 600 python bench.py $(bench_args "${s#bench_}" | sed 's/--no-cpu-baseline//') ;;
    benchn_*) run "$s" 600 python bench.py $(bench_args "${s#benchn_}") ;;
    cold_*) C=${s#cold_}; K=20; [ "${C%_k*}" != "$C" ] && K=${C##*_k} && C=${C%_k*}
      run "$s" 600 python bench.py --config "$C" --cache cold --steps "$K" --no-cpu-baseline ;;
    prof_*) C=${s#prof_}
      run "$s" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$s" -o run \
        -- python bench.py $(bench_args "$C") ;;
    pmc_*) C=${s#pmc_}
      run "pmc_fetch_$C" 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$C" \
        -o run -- python bench.py $(bench_args "$C")
      run "pmc_write_$C" 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$C" \
        -o run -- python bench.py $(bench_args "$C") ;;
    sq_*) C=${s#sq_}
      run "$s" 180 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/$s" -o run \
        -- python bench.py $(bench_args "$C") ;;
    kurtsq_*) C=${s#kurtsq_}
      run "$s" 180 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/$s" -o run \
        -- python bench.py --mode kurtosis --config "$C" --steps 20 --warmup 5 ;;
    gloo_*)  # N ranks sharing the one GPU over gloo (the driver's N-GPU path, exchange and
             # self-check included; REHEARSAL, not a scaling number): gloo_N_CFG
      A=${s#gloo_}; N=${A%%_*}; C=${A#*_}
      run "$s" 600 python bench.py --gpus "$N" --dist-backend gloo --config "$C" --steps 10 \
        --warmup 3 --no-cpu-baseline ;;
    kurtsweep)  # k_kurt_i8's grid knobs: waves per CU x shortest slab
      for W in ${KS_W:-12 16 24 32}; do for S in ${KS_S:-16 32 64}; do
        BLDP_KURT_I8_WAVES_PER_CU=$W BLDP_KURT_I8_MIN_SLAB=$S run "kurtsweep_w${W}_s$S" 300 \
          python tools/ab_variants.py --run --suite typedk --rounds 3 --variants base \
          --json "$OUT/kurtsweep_w${W}_s$S.json"
      done; done ;;
    ab_*) A=${s#ab_}; SUITE=${A%%:*}; V=${AB_VARIANTS:-base}; [ "$SUITE" != "$A" ] && V=${A#*:}
      run "ab_$SUITE" 900 python tools/ab_variants.py --run --suite "$SUITE" --rounds 5 \
          --variants "$V" --json "$OUT/ab_$SUITE.json" ;;
    kurt_*) run "$s" 300 python bench.py --mode kurtosis --config "${s#kurt_}" ;;
    ceil_kurt) run ceil_kurt 600 ./build/mix_ceiling 10 kurt ;;
    hostbound) run hostbound 600 python tools/host_bound_probe.py --json "$OUT/hostbound.json" ;;
    kurtprof_*) C=${s#kurtprof_}
      run "$s" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$s" -o run \
        -- python bench.py --mode kurtosis --config "$C" --steps 20 --warmup 5 ;;
    kurtpmc_*) C=${s#kurtpmc_}
      run "kurtpmc_fetch_$C" 180 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d "$OUT/kurtpmc_fetch_$C" -o run -- python bench.py --mode kurtosis --config "$C" \
        --steps 20 --warmup 5
      run "kurtpmc_write_$C" 180 rocprofv3 --pmc WRITE_SIZE --output-format csv \
        -d "$OUT/kurtpmc_write_$C" -o run -- python bench.py --mode kurtosis --config "$C" \
        --steps 20 --warmup 5 ;;
    file) run file 300 python bench.py --mode file ;;
    rawfile) run rawfile 300 python bench.py --mode rawfile ;;
    typed) run typed 300 python bench.py --mode typed ;;
    typedw_*) W=${s#typedw_}; BLDP_KURT_I8_WAVES_PER_CU=$W run "$s" 300 python bench.py --mode typed ;;
    typedwarm) run typedwarm 300 python bench.py --mode typed --cache warm ;;
    typedpipe_*) run "$s" 300 python bench.py --mode typed --plan-option typed_pipe="${s#typedpipe_}" ;;
    typedprof) run typedprof 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/typedprof" -o run -- python bench.py --mode typed --steps 20 --warmup 5 ;;
    typedpmc)
      run typedpmc_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/typedpmc_fetch" \
        -o run -- python bench.py --mode typed --steps 20 --warmup 5
      run typedpmc_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/typedpmc_write" \
        -o run -- python bench.py --mode typed --steps 20 --warmup 5 ;;
    typedsq) run typedsq 180 rocprofv3 --pmc $SQ --output-format csv -d "$OUT/typedsq" -o run \
        -- python bench.py --mode typed --steps 20 --warmup 5 ;;
    getband) run getband 600 python tools/getband_probe.py --json "$OUT/getband.json" ;;
    dist*) N=${s#dist}; run "$s" 400 python bench.py --gpus "$N" --dist-backend gloo --steps 5 \
        --warmup 2 --no-cpu-baseline ;;
    probe_cold) run probe_cold 300 python tools/hbm_probe.py 68.07 156.99 557.5 --cold ;;
    getbandz) run getbandz 600 python tools/getband_probe.py --compressed --json "$OUT/getbandz.json" ;;
    getband_t*) run "$s" 600 python tools/getband_probe.py --threads "${s#getband_t}" \
        --cases "F64 T1,F1 T1 despike" --json "$OUT/$s.json" ;;
    getbandb_*) IFS=_ read -r B R T X <<< "${s#getbandb_}"  # getbandb_BATCHMB_RINGMB_THREADS[_rep]
      run "$s" 300 python tools/getband_probe.py --threads "$T" --batch-mb "$B" --ring-mb "$R" \
        --cases "F64 T1" --json "$OUT/$s.json" ;;
    getbandzp) run getbandzp 600 python tools/getband_probe.py --compressed \
        --cases "F64 T1" --json "$OUT/getbandzp.json" ;;
  esac
done
echo "== session done"
