#!/bin/bash
# Round 5: bench.py --mode rawfile (one 2 GiB uncompressed FBH5 file, getdata
# end to end) with the old reader setup against the NUMA-node defaults,
# alternating on one box.
set -u
O=gpurun_out/${1:-r05y}; mkdir -p $O
for i in 1 2 3 4; do
  for c in old new; do
    if [ $c = old ]; then export BLDP_READ_AFFINITY=0 BLDP_SLOT_NUMA=0 BLDP_READ_THREADS=16
    else unset BLDP_READ_AFFINITY BLDP_SLOT_NUMA BLDP_READ_THREADS; fi
    timeout -k 10 300 python bench.py --mode rawfile --no-cpu-baseline > $O/rawfile_${c}_$i.log 2>&1 \
      || { echo "rawfile $c $i failed"; exit 1; }
    echo "${c}_$i $(grep -o '"value": [0-9.]*' $O/rawfile_${c}_$i.log | head -1)"
  done
done
