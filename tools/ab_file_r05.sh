#!/bin/bash
# Round 5: compressed reads staged through the pinned slot ring (8 or 16 x 32
# MiB) against the round-5 build that staged each window in one pinned buffer
# (build/prevtree), alternating on one box: bench.py --mode file (one 1 GiB
# file) and tools/getband_probe.py --compressed (8 files, 476 MB stored).
# build/prevtree: `git archive <rev> bench.py __graft_entry__.py
# bldistributeddataproducts.jl_amd tools/getband_probe.py tests/golden | tar -x
# -C build/prevtree`, plus oracle/ and that revision's built libbldp_hip.so.
set -u
O=gpurun_out/${1:-r05m}; mkdir -p $O
R=$PWD
for i in 1 2 3; do
  for t in ring8 prev ring16; do
    D=$R; E=""
    [ $t = prev ] && D=$R/build/prevtree
    [ $t = ring16 ] && E="BLDP_RING_SLOTS=16 BLDP_NATIVE_RING_MB=512"
    (cd $D && env $E timeout -k 10 300 python bench.py --mode file --no-cpu-baseline > $R/$O/file_${t}_$i.log 2>&1) || { echo "file $t $i failed"; exit 1; }
    (cd $D && env $E timeout -k 10 300 python tools/getband_probe.py --compressed --cases "F64 T1" --json $R/$O/getbandz_${t}_$i.json > $R/$O/getbandz_${t}_$i.log 2>&1) || { echo "getbandz $t $i failed"; exit 1; }
    echo "$t $i: file $(grep -o '"value": [0-9.]*' $R/$O/file_${t}_$i.log | head -1) getbandz $(grep -o '"device": {"median_ms": [0-9.]*' $R/$O/getbandz_${t}_$i.log)"
  done
done
