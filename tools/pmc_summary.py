"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel (HBM traffic per launch).

FETCH_SIZE and WRITE_SIZE are reported in KiB per dispatch. MI355X_MICROARCH.md (HBM section): on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read, so it is doubled here; WRITE_SIZE is taken as is.

    python tools/pmc_summary.py gpurun_out/pmc_fetch/bench_counter_collection.csv \
        gpurun_out/pmc_write/bench_counter_collection.csv > profiles/rNN/pmc_summary.json
"""
import csv
import json
import sys
from collections import defaultdict


def short(name: str) -> str:
    return name.split("(")[0].replace("ccmi::", "")


def load(path: str):
    acc = defaultdict(lambda: [0, 0.0])
    counter = None
    with open(path) as f:
        for row in csv.DictReader(f):
            counter = row["Counter_Name"]
            a = acc[short(row["Kernel_Name"])]
            a[0] += 1
            a[1] += float(row["Counter_Value"])
    return counter, acc


def main():
    out = {"note": "bytes per launch; FETCH_SIZE doubled (gfx950 correction), WRITE_SIZE as reported",
           "kernels": {}}
    for path in sys.argv[1:]:
        counter, acc = load(path)
        scale = 2.0 if counter == "FETCH_SIZE" else 1.0
        for k, (n, kib) in acc.items():
            d = out["kernels"].setdefault(k, {})
            d["launches"] = n
            d[f"{counter.lower()}_bytes_per_launch"] = kib * 1024.0 * scale / n
    for d in out["kernels"].values():
        d["hbm_bytes_per_launch"] = d.get("fetch_size_bytes_per_launch", 0.0) + d.get("write_size_bytes_per_launch", 0.0)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
