#!/bin/bash
# Round 3, the reference's own fqav (tavby = 1): read:write-mix ceilings,
# A/B of library variants on the VERDICT r02 shapes, kernel stats and PMC
# passes (one counter group per run, MI355X_MICROARCH.md §rocprofv3 PMC slots).
#   usage: tools/r03_t1_session.sh TAG [steps...]   steps: mix tests tests_K smoke ab stats pmc
# Every GPU step has its own time limit; after a failure nothing more runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03a}; shift || true
STEPS=${*:-"mix ab stats pmc"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "== $name failed (rc=$rc): stopping GPU work"; exit $rc; fi
}

pmc() {  # name counters...
  local name=$1; shift
  run "pmc_$name" 180 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/pmc_$name" -o run \
    -- python tools/t1_probe.py --pmc --which "${T1_WHICH:-all}" --json "$OUT/cases.json"
}

for s in $STEPS; do
  case $s in
    mix) run mix 300 ./build/mix_ceiling 10 ;;
    mixdword) run mixdword 120 ./build/mix_ceiling 10 dword ;;
    coltile) run coltile 120 ./build/mix_ceiling 10 coltile ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
          --timeout-method thread ;;
    tests_*) run "$s" 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
          --timeout-method thread -k "${s#tests_}" ;;
    getband) run getband 600 python tools/getband_probe.py --json "$OUT/getband.json" ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as e; e.smoke()" ;;
    ab) run ab 900 python tools/ab_variants.py --run --suite t1v --rounds 5 \
          --variants "${AB_VARIANTS:-base,dpp,r02}" --json "$OUT/ab_t1v.json" ;;
    ab_*) run "$s" 900 python tools/ab_variants.py --run --suite "${s#ab_}" --rounds 5 \
          --variants "${AB_VARIANTS:-base,r02}" --json "$OUT/$s.json" ;;
    stats) run stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run \
          -- python tools/t1_probe.py --rounds 3 --iters 10 --which "${T1_WHICH:-all}" \
          --json "$OUT/t1_probe.json" ;;
    pmc)
      pmc fetch FETCH_SIZE
      pmc write WRITE_SIZE
      pmc tccreq TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
      pmc tccstall TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum \
        TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum
      pmc sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT
      pmc sqmem SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_WR \
        SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS
      ;;
  esac
done
echo "== session done"
