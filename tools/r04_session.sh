#!/bin/bash
# Round 4 GPU sessions: per-config kernel stats and PMC passes (one counter
# group per run, MI355X_MICROARCH.md §rocprofv3), A/B suites, tests, bench.
#   usage: tools/r04_session.sh TAG [steps...]
#   steps: smoke tests tests_K bench bench_CFG prof_CFG pmc_CFG sq_CFG ab_SUITE mix1 typed typedprof gap getband
# Every GPU step has its own time limit; after any failure nothing more runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r04a}; shift || true
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
  tail -n 6 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "== $name failed (rc=$rc): stopping GPU work"; exit $rc; fi
}

bench_args() {  # CFG -> bench.py arguments for a short profiled run
  echo "--config $1 --steps 20 --warmup 5 --no-cpu-baseline"
}

for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as e; e.smoke()" ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
          --timeout-method thread ;;
    tests_*) run "$s" 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
          --timeout-method thread -k "${s#tests_}" ;;
    bench) run bench 600 python bench.py ;;
    bench_*) run "$s" 600 python bench.py --config "${s#bench_}" ;;
    benchw_*) run "$s" 600 python bench.py --config "${s#benchw_}" --warmup 300 --no-cpu-baseline ;;
    prof_*) C=${s#prof_}
      run "$s" 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$s" -o run \
        -- python bench.py $(bench_args "$C") ;;
    pmc_*) C=${s#pmc_}
      run "pmc_fetch_$C" 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$C" \
        -o run -- python bench.py $(bench_args "$C")
      run "pmc_write_$C" 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$C" \
        -o run -- python bench.py $(bench_args "$C") ;;
    sq_*) C=${s#sq_}
      run "$s" 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT \
        --output-format csv -d "$OUT/$s" -o run -- python bench.py $(bench_args "$C")
      run "${s}_tcc" 180 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum \
        TCC_EA0_RDREQ_32B_sum --output-format csv -d "$OUT/${s}_tcc" -o run \
        -- python bench.py $(bench_args "$C") ;;
    ab_*) run "$s" 900 python tools/ab_variants.py --run --suite "${s#ab_}" --rounds 5 \
          --variants "${AB_VARIANTS:-base}" --json "$OUT/$s.json" ;;
    mix1) run mix1 300 ./build/mix_ceiling 10 0001 ;;
    mix2) run mix2 300 ./build/mix_ceiling 10 0002 ;;
    typed) run typed 300 python bench.py --mode typed ;;
    typed_*) run "$s" 300 python bench.py --mode typed --plan-option typed_rows="${s#typed_}" ;;
    typedoff) run typedoff 300 python bench.py --mode typed --plan-option typed_vec=0 ;;
    typedprof) run typedprof 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/typedprof" -o run -- python bench.py --mode typed --steps 20 --warmup 5 ;;
    gap) run gap 300 python tools/gap_probe.py --json "$OUT/gap.json" ;;
    getband64) run getband64 600 env BLDP_NATIVE_BATCH_MB=64 python tools/getband_probe.py \
        --json "$OUT/getband64.json" ;;
    probesweep) run probesweep 300 python tools/read_probe_sweep.py --json "$OUT/probesweep.json" ;;
    getband) run getband 600 python tools/getband_probe.py --json "$OUT/getband.json" ;;
  esac
done
echo "== session done"
