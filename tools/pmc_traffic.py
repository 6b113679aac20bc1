"""Per-launch HBM traffic of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE),
corrected as MI355X_MICROARCH.md §HBM prescribes: both counters are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced read, so it is doubled.

usage: python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv>
                                   <kernel-substring> <out.json> [round] [batch]
The record carries the workload (bench.py defaults) and the sha1 of the library build it measured,
so bench.py only reports it for that exact build.
"""
import csv
import json
import sys


def per_dispatch(path, counter, kernel):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fpath, wpath, kernel, out = sys.argv[1:5]
    rnd = sys.argv[5] if len(sys.argv) > 5 else "r01"
    batch = int(sys.argv[6]) if len(sys.argv) > 6 else 1308  # bench.py's default on MI355X (256 CUs, T=100; 327 before round 5)
    profile = sys.argv[7] if len(sys.argv) > 7 else "default"  # world profile of the measured batch
    fetch = per_dispatch(fpath, "FETCH_SIZE", kernel)
    write = per_dispatch(wpath, "WRITE_SIZE", kernel)
    if not fetch or not write:
        raise SystemExit(f"no {kernel} rows in {fpath} / {wpath}")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    res = dict(kernel=kernel, launches=[len(fetch), len(write)], fetch_size_kib=f_kib, write_size_kib=w_kib,
               traffic_bytes_per_launch=(2 * f_kib + w_kib) * 1024,
               correction="bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md HBM)",
               config=dict(T=100, O=20, batch=batch), profile=profile, round=rnd,
               command=f"rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE --output-format csv -- python3 bench.py --batch {batch} "
                       "--steps 1 --warmup 0 --cpu-seconds 0 --no-extras (tools/gpu.sh traffic)")
    import hashlib
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "armour-dev_amd", "armour_amd", "libarmour_hip.so")
    res["lib_sha1"] = hashlib.sha1(open(lib, "rb").read()).hexdigest()[:16]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
