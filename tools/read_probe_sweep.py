#!/usr/bin/env python3
"""The pure-read probe (tools/hbm_probe.hip) over grid forms and buffer sizes:
which form bench.py's box reference should try.

    python tools/read_probe_sweep.py [--json out.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="68,272,545,1090,4096,32768")
    ap.add_argument("--wg", default="0,1,2,3,4,8")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import hbm_probe
    forms = tuple(m << 8 | int(g) for m in (0, 1, 2, 3, 4, 5, 6, 7) for g in a.wg.split(","))
    res = {}
    for mb in (int(m) for m in a.sizes_mb.split(",")):
        r = hbm_probe.read_probe(mb << 20, launches=20, forms=forms, every=True)
        res[mb] = r
        print(mb, "MiB best", r["GBps"], "at form", r["form"], flush=True)
        for f in r["forms"]:
            print(f"   wg/cu {f['wg_per_cu']:2d} {f['loads']:5s} {f['in_flight']:2d} in flight "
                  f"{'slabs' if f['slabs'] else 'contig'}: "
                  f"{f['GBps']}", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
