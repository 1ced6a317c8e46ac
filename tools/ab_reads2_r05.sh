#!/bin/bash
# Round 5: the reads A/B with more alternations (raw and compressed getband
# only, F64 T1): the old reader setup (16 threads anywhere, slots wherever the
# runtime puts them) against the defaults (NUMA-node readers and slots,
# threads from the CPU quota).
set -u
O=gpurun_out/${1:-r05w}; mkdir -p $O
cat /sys/bus/pci/devices/*/numa_node > /dev/null 2>&1
python - <<'PY' > $O/node.txt 2>&1 || true
import ctypes, torch
torch.cuda.init()
print("gpu pci", torch.cuda.get_device_properties(0).pci_bus_id if hasattr(torch.cuda.get_device_properties(0), "pci_bus_id") else "?")
PY
for i in 1 2 3 4 5 6; do
  for c in old new; do
    n=${c}_$i
    if [ $c = old ]; then export BLDP_READ_AFFINITY=0 BLDP_SLOT_NUMA=0 BLDP_READ_THREADS=16
    else unset BLDP_READ_AFFINITY BLDP_SLOT_NUMA BLDP_READ_THREADS; fi
    timeout -k 10 300 python tools/getband_probe.py --reps 7 --cases "F64 T1" --json $O/raw_$n.json \
      > $O/raw_$n.log 2>&1 || { echo "raw $n failed"; exit 1; }
    timeout -k 10 300 python tools/getband_probe.py --reps 7 --compressed --cases "F64 T1" \
      --json $O/z_$n.json > $O/z_$n.log 2>&1 || { echo "z $n failed"; exit 1; }
    echo "$n raw $(grep -o '"device": {"median_ms": [0-9.]*' $O/raw_$n.log | grep -o '[0-9.]*$') z $(grep -o '"device": {"median_ms": [0-9.]*' $O/z_$n.log | grep -o '[0-9.]*$')"
  done
done
