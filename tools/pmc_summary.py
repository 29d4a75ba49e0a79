"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel (HBM traffic per launch).

FETCH_SIZE and WRITE_SIZE are reported in KiB per dispatch. MI355X_MICROARCH.md (HBM section): on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced (16 B/lane) read and WRITE_SIZE is exact for 16 B/lane
stores; other access widths must be calibrated on a known byte count in the kernel's own access pattern.

Two modes:

    # 1. calibration: pair tools/pmc_calib's known byte counts with its counter passes
    python tools/pmc_summary.py --calib calib_bytes.json calib_FETCH*.csv calib_WRITE*.csv > calib_summary.json
    # 2. a workload: per-kernel bytes, each kernel scaled by the factor of the calibration pattern it matches
    #    (CALIB_PATTERN below; uncalibrated kernels keep the guide's x2 FETCH / x1 WRITE)
    python tools/pmc_summary.py --calib calib_summary.json fetch.csv write.csv > profiles/rNN/c2_pmc_summary.json
"""
import csv
import json
import sys
from collections import defaultdict

# Which calibration kernel's access pattern each product kernel follows. scan_* / chain_* read destination
# BrokerRecs (128 B) and ReplicaRec / PartitionRec (64 B) rows at scattered indices, one record per lane; stats_topics
# streams topicCount rows 16 B per lane.
CALIB_PATTERN = {
    "scan_cross": "gather128", "scan_pairs": "gather128", "scan_swap": "gather128", "chain_pairs": "gather128",
    "chain_rack_rows": "gather128", "stats_topics": "stream16",
}
DEFAULT_FACTOR = {"FETCH_SIZE": 2.0, "WRITE_SIZE": 1.0}


def short(name: str) -> str:
    return name.split("(")[0].replace("ccmi::", "").replace("void ", "").strip()


def load(path: str):
    """counter name, {kernel: [dispatch KiB values in file order]}"""
    acc = defaultdict(list)
    counter = None
    with open(path) as f:
        for row in csv.DictReader(f):
            counter = row["Counter_Name"]
            acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return counter, acc


def calibrate(known_path, csvs):
    with open(known_path) as f:
        known = json.load(f)
    out = {"note": "factor = known bytes / counter bytes (raw KiB x 1024), last dispatch of each kernel; table "
                   f"{known['table_bytes']} B, 4x the Infinity Cache", "kernels": {}, "factors": {}}
    for path in csvs:
        counter, acc = load(path)
        field = "read" if counter == "FETCH_SIZE" else "write"
        for k, vals in acc.items():
            if k not in known["kernels"]:
                continue
            raw = vals[-1] * 1024.0
            kb = known["kernels"][k][field]
            d = out["kernels"].setdefault(k, {})
            d[f"{counter.lower()}_raw_bytes"] = raw
            d[f"known_{field}_bytes"] = kb
            f_ = kb / raw if raw > 0 else None
            d[f"{counter.lower()}_factor"] = f_
            out["factors"].setdefault(k, {})[counter] = f_
    return out


def summarise(calib_path, csvs):
    factors = {}
    if calib_path:
        with open(calib_path) as f:
            factors = json.load(f)["factors"]
    out = {"note": "bytes per launch; each counter scaled by the calibration factor of the kernel's access pattern "
                   "(calibration), else x2 FETCH_SIZE / x1 WRITE_SIZE (MI355X_MICROARCH.md)",
           "calibration": calib_path, "kernels": {}}
    for path in csvs:
        counter, acc = load(path)
        for k, vals in acc.items():
            pat = CALIB_PATTERN.get(k)
            scale = factors.get(pat, {}).get(counter) if pat else None
            src = pat if scale else "guide default"
            scale = scale or DEFAULT_FACTOR[counter]
            d = out["kernels"].setdefault(k, {})
            d["launches"] = len(vals)
            d[f"{counter.lower()}_raw_bytes_per_launch"] = sum(vals) * 1024.0 / len(vals)
            d[f"{counter.lower()}_bytes_per_launch"] = sum(vals) * 1024.0 * scale / len(vals)
            d[f"{counter.lower()}_scale"] = {"factor": scale, "source": src}
    for d in out["kernels"].values():
        d["hbm_bytes_per_launch"] = d.get("fetch_size_bytes_per_launch", 0.0) + d.get("write_size_bytes_per_launch", 0.0)
    return out


def main():
    args = sys.argv[1:]
    calib = None
    if args and args[0] == "--calib":
        calib, args = args[1], args[2:]
    if calib:
        with open(calib) as f:
            is_known = "table_bytes" in json.load(f)
        out = calibrate(calib, args) if is_known else summarise(calib, args)
    else:
        out = summarise(None, args)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
