#!/bin/bash
# Round 5: reader threads confined to the GPU's NUMA node (BLDP_READ_AFFINITY),
# pinned slots placed on that node (BLDP_SLOT_NUMA) and the reader count,
# alternating on one box: GBT.getband of 8 page-cached raw 0002 files and of 8
# compressed ones (tools/getband_probe.py, F64 T1), and bench.py --mode file.
# Configurations a_m_t (affinity, slot placement, threads; "d" = the default).
set -u
O=gpurun_out/${1:-r05t}; mkdir -p $O
CONFIGS=${2:-"0_0_16 d_d_d"}
for i in 1 2 3; do
  for c in $CONFIGS; do
    IFS=_ read -r a m t <<< "$c"
    n=c${c}_$i
    unset BLDP_READ_AFFINITY BLDP_SLOT_NUMA BLDP_READ_THREADS
    [ "$a" != d ] && export BLDP_READ_AFFINITY=$a
    [ "$m" != d ] && export BLDP_SLOT_NUMA=$m
    [ "$t" != d ] && export BLDP_READ_THREADS=$t
    timeout -k 10 300 python tools/getband_probe.py --cases "F64 T1" --json $O/raw_$n.json \
      > $O/raw_$n.log 2>&1 || { echo "raw $n failed"; exit 1; }
    timeout -k 10 300 python tools/getband_probe.py --compressed --cases "F64 T1" \
      --json $O/z_$n.json > $O/z_$n.log 2>&1 || { echo "z $n failed"; exit 1; }
    timeout -k 10 300 python bench.py --mode file --no-cpu-baseline > $O/file_$n.log 2>&1 \
      || { echo "file $n failed"; exit 1; }
    echo "$n raw $(grep -o '"device": {"median_ms": [0-9.]*' $O/raw_$n.log | grep -o '[0-9.]*$') z $(grep -o '"device": {"median_ms": [0-9.]*' $O/z_$n.log | grep -o '[0-9.]*$') file $(grep -o '"value": [0-9.]*' $O/file_$n.log | head -1 | grep -o '[0-9.]*$') threads $(grep -o '"threads": [0-9]*' $O/raw_$n.log | head -1 | grep -o '[0-9]*$')"
  done
done
