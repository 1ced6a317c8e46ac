#!/bin/bash
# One GPU session on the MI355X box: probe, smoke, GPU parity tests, bench,
# rocprofv3 kernel stats.  Every GPU step has its own time limit; after a
# crash/abort/timeout nothing further touches the GPU.
#   usage: tools/gpu_session.sh TAG [steps...]   steps: smoke tests bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}; shift || true
STEPS=${*:-"smoke tests bench prof"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 12 "$OUT/$name.log"
  case $rc in
    0|1) return 0 ;;   # 1 = test/assert failures: the GPU is fine
    *) echo "== $name ended with rc=$rc: stopping GPU work"; exit $rc ;;
  esac
}

{ which julia || echo "julia: absent"; rocm-smi --showproductname 2>/dev/null | head -8; nproc; } \
  > "$OUT/probe.log" 2>&1
for s in $STEPS; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as e; e.smoke()" ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    bench) run bench 600 python bench.py ;;
    prof)  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/prof" -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv \
             -d "$OUT/pmc_fetch" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv \
             -d "$OUT/pmc_write" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    pmclb_*) K=${s#pmclb_}
           run "pmc_fetch_lb$K" 300 rocprofv3 --pmc FETCH_SIZE --output-format csv \
             -d "$OUT/pmc_fetch_lb$K" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --local-banks "$K"
           run "pmc_write_lb$K" 300 rocprofv3 --pmc WRITE_SIZE --output-format csv \
             -d "$OUT/pmc_write_lb$K" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --local-banks "$K" ;;
    benchlb_*) run "$s" 300 python bench.py --no-cpu-baseline --local-banks "${s#benchlb_}" ;;
    bench_*) run "$s" 600 python bench.py --config "${s#bench_}" ;;
    benchperbank) run benchperbank 600 python bench.py --band-alloc per-bank --no-cpu-baseline ;;
    benchnocpu) run benchnocpu 600 python bench.py --no-cpu-baseline ;;
    kurt_*) run "$s" 600 python bench.py --mode kurtosis --config "${s#kurt_}" ;;
    host)  run host 900 python bench.py --mode host ;;
    host2) run host2 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
             --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 2 --dist-backend gloo \
             --mode host ;;
    decode) run decode 600 python bench.py --mode decode ;;
    file)  run file 600 python bench.py --mode file ;;
    file_probe) run file_probe 600 python tools/file_probe.py ;;
    rawfile) run rawfile 600 python bench.py --mode rawfile ;;
    rawfile_ring) BLDP_PAGECACHE_DMA=0 run rawfile_ring 600 python bench.py --mode rawfile ;;
    rawtests) run rawtests 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "raw or fil or gbt" ;;
    rawfile_py) BLDP_NATIVE_READ=0 run rawfile_py 600 python bench.py --mode rawfile ;;
    file_py) BLDP_NATIVE_READ=0 run file_py 600 python bench.py --mode file ;;
    paths) run paths 300 python tools/probe_paths.py ;;
    paths_big) run paths_big 300 python tools/probe_paths.py --big ;;
    prof_paths) run prof_paths 300 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/prof_paths" -o run -- python tools/probe_paths.py --big
           run pmc_fetch_paths 300 rocprofv3 --pmc FETCH_SIZE --output-format csv \
             -d "$OUT/pmc_fetch_paths" -o run -- python tools/probe_paths.py --big
           run pmc_write_paths 300 rocprofv3 --pmc WRITE_SIZE --output-format csv \
             -d "$OUT/pmc_write_paths" -o run -- python tools/probe_paths.py --big ;;
    prof_decode) run prof_decode 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/prof_decode" -o run -- python bench.py --mode decode ;;
    prof_kurt) run prof_kurt 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/prof_kurt" -o run -- python bench.py --mode kurtosis --config cfg3 ;;
    prof_kurt_*) run "$s" 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d "$OUT/$s" -o run -- python bench.py --mode kurtosis --config "${s#prof_kurt_}" ;;
    pmc_kurt_*) C=${s#pmc_kurt_}
           run "pmc_fetch_kurt_$C" 300 rocprofv3 --pmc FETCH_SIZE --output-format csv \
             -d "$OUT/pmc_fetch_kurt_$C" -o run -- python bench.py --mode kurtosis --config "$C" --steps 5 --warmup 2
           run "pmc_write_kurt_$C" 300 rocprofv3 --pmc WRITE_SIZE --output-format csv \
             -d "$OUT/pmc_write_kurt_$C" -o run -- python bench.py --mode kurtosis --config "$C" --steps 5 --warmup 2 ;;
    dist2) run dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
             --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --dist-backend gloo \
             --steps 10 --warmup 3 ;;
    dist4|dist8) run "$s" 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "${s#dist}" \
             --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus "${s#dist}" --dist-backend gloo \
             --steps 10 --warmup 3 ;;
    dist2c2) run dist2c2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
             --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --dist-backend gloo \
             --steps 10 --warmup 3 --config cfg2 ;;
    unal_check) run unal_check 300 python tools/unaligned_check.py --variant "${UNAL_VARIANT:-unal2}" ;;
    nmix)  run nmix 300 ./build/hbm_ceiling 32 10 bldistributeddataproducts.jl_amd/libbldp_hip.so nmix ;;  # (built here: hipcc -o build/hbm_ceiling tools/hbm_ceiling.hip -ldl)
    pipeline) run pipeline 600 python bench.py --pipeline --no-cpu-baseline ;;
    prof_pipelb_*) run "$s" 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$s" -o run \
             -- python bench.py --pipeline --no-cpu-baseline --local-banks "${s#prof_pipelb_}" --steps 20 --warmup 5 ;;
    stream_probe) run stream_probe 300 python tools/stream_probe.py ;;
    stream_probe_hi) TORCH_NCCL_HIGH_PRIORITY=1 run stream_probe_hi 300 python tools/stream_probe.py --variants none,torch_async,torch_side ;;
    prof_bench_pipe) run prof_bench_pipe 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$s" -o run \
             -- python bench.py --pipeline --no-cpu-baseline --local-banks 1 --steps 20 --warmup 5 ;;
    prof_stream_probe) run prof_stream_probe 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$s" -o run \
             -- python tools/stream_probe.py --steps 20 --warmup 5 ;;
    pipelb_*) run "$s" 300 python bench.py --pipeline --no-cpu-baseline --local-banks "${s#pipelb_}" --steps 50 --warmup 10 ;;
    ab)    run ab 900 python tools/ab_variants.py --run --variants "${AB_VARIANTS:-base,noil}" --json "$OUT/ab.json" ;;
    ab_kurt) run ab_kurt 900 python tools/ab_variants.py --run --suite kurt --variants ${AB_VARIANTS:-base,kold,kw5,kw6} --json "$OUT/ab_kurt.json" ;;
    ab_kleaf) run ab_kleaf 600 python tools/ab_variants.py --run --suite kleaf --variants "${AB_VARIANTS:-base,kleafb2,kleafpipe2,kleafpipe2w5}" --json "$OUT/ab_kleaf.json" ;;
    mmap_probe) run mmap_probe 300 python tools/mmap_register_probe.py ;;
    ab_kmid) run ab_kmid 600 python tools/ab_variants.py --run --suite kmid --variants "${AB_VARIANTS:-base,kmid2w8,kmid2w4}" --json "$OUT/ab_kmid.json" ;;
    ab_row) run ab_row 600 python tools/ab_variants.py --run --suite row --variants "${AB_VARIANTS:-base,rowmw3,rowmw5,rowmw6}" --json "$OUT/ab_row.json" ;;
    ab_t1) run ab_t1 600 python tools/ab_variants.py --run --suite t1 --variants "${AB_VARIANTS:-base,norowt}" --json "$OUT/ab_t1.json" ;;
    sweep) run sweep 600 python tools/ab_variants.py --run --suite sweep --rounds 3 --variants "${AB_VARIANTS:-base}" --json "$OUT/sweep.json" ;;
    ab_il1) run ab_il1 600 python tools/ab_variants.py --run --suite il1 --variants "${AB_VARIANTS:-base,wavet2}" --json "$OUT/ab_il1.json" ;;
    counters) run counters 60 rocprofv3 -L ;;
    sq_kurt_*) run "$s" 120 rocprofv3 --pmc ${SQC:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT} \
             --output-format csv -d "$OUT/$s" -o run -- python bench.py --mode kurtosis --config "${s#sq_kurt_}" --steps 5 --warmup 2 ;;
    sq_red_*) run "$s" 120 rocprofv3 --pmc ${SQC:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT} \
             --output-format csv -d "$OUT/$s" -o run -- python bench.py --config "${s#sq_red_}" --steps 5 --warmup 2 --no-cpu-baseline ;;
    ab_tile) run ab_tile 900 python tools/ab_variants.py --run --suite tile --variants "${AB_VARIANTS:-base,tk4a1,tk2a1,tk2a2}" --json "$OUT/ab_tile.json" ;;
  esac
done
echo "== session done"
