#!/bin/bash
# Round 5: the raw reader's ramped batches (slot/4, slot/2 ... slot/2, slot/4)
# against slot-sized ones (BLDP_RUNS_RAMP=0), alternating on one box: GBT.getband
# of 8 raw 0002 files (F64 T1) and bench.py --mode rawfile (one 2 GiB file).
set -u
O=gpurun_out/${1:-r05z}; mkdir -p $O
for i in 1 2 3 4; do
  for r in 0 1; do
    n=ramp${r}_$i
    BLDP_RUNS_RAMP=$r timeout -k 10 300 python tools/getband_probe.py --reps 7 --cases "F64 T1" \
      --json $O/raw_$n.json > $O/raw_$n.log 2>&1 || { echo "raw $n failed"; exit 1; }
    BLDP_RUNS_RAMP=$r timeout -k 10 300 python bench.py --mode rawfile --no-cpu-baseline \
      > $O/rawfile_$n.log 2>&1 || { echo "rawfile $n failed"; exit 1; }
    echo "$n raw $(grep -o '"device": {"median_ms": [0-9.]*' $O/raw_$n.log | grep -o '[0-9.]*$') read_call $(grep -o '"read_call_ms": [0-9.]*' $O/raw_$n.log | head -1 | grep -o '[0-9.]*$') first $(grep -o '"first_copy_ms": [0-9.]*' $O/raw_$n.log | head -1 | grep -o '[0-9.]*$') rawfile $(grep -o '"value": [0-9.]*' $O/rawfile_$n.log | head -1 | grep -o '[0-9.]*$')"
  done
done
