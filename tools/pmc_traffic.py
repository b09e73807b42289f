"""HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE CSVs
(separate passes, as /opt/skills/guides/MI355X_MICROARCH.md prescribes).

FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters, TCC EA
requests). gfx950 correction from the guide: FETCH_SIZE reports half of the
bytes of wide coalesced 16-B/lane reads (TCC_EA0_RDREQ x 64 B for 128-B
requests); it is applied here to the read side, which makes the read figure
an upper bound for narrower accesses. WRITE_SIZE is taken as is.

    python tools/pmc_traffic.py gpurun_out/<tag> > profiles/pmc_readme_1920x1080_s8x8.json
"""
import csv
import json
import os
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"]
            short = name.replace("void ", "").replace("(anonymous namespace)::", "")
            short = short.split("(")[0].split("<")[0].split("::")[-1]
            acc[(short, row["Dispatch_Id"])].append(float(row["Counter_Value"]))
    out = defaultdict(list)
    for (short, _), vals in acc.items():
        out[short].append(sum(vals))
    return {k: sum(v) / len(v) for k, v in out.items()}


def main(d):
    fetch = per_kernel(os.path.join(d, "pmc_fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(d, "pmc_write", "write_counter_collection.csv"), "WRITE_SIZE")
    build = None   # the library build the passes ran: profile_round.sh's bench.json of the same directory
    try:
        with open(os.path.join(d, "bench.json")) as f:
            build = json.loads(f.read().strip().splitlines()[-1]).get("build_id")
    except (OSError, ValueError, IndexError):
        pass
    res = {"source": d, "build_id": build, "units": "bytes per launch (dispatch mean)",
           "correction": "read = 2 x FETCH_SIZE KiB x 1024 (gfx950 half-count of 128-B requests); write = WRITE_SIZE KiB x 1024"}
    for k in sorted(set(fetch) | set(write)):
        if k.startswith("__amd") or "elementwise" in k:
            continue
        rd = 2 * fetch.get(k, 0.0) * 1024
        wr = write.get(k, 0.0) * 1024
        res[k] = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes_per_launch": rd + wr}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
