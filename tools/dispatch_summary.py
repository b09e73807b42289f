"""Per-dispatch durations, scratch and VGPRs of every kernel in a rocprofv3
--kernel-trace CSV (tools/profile_round.sh writes <tag>/ks/ks_kernel_trace.csv).

    python tools/dispatch_summary.py gpurun_out/<tag> > profiles/r02/kernel_dispatches_<name>.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    s = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return s.split("(")[0]


def main(tag_dir):
    path = glob.glob(os.path.join(tag_dir, "ks", "*kernel_trace.csv"))[0]
    ms = defaultdict(list)
    scratch, vgpr, lds = {}, {}, {}
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            if k.startswith("__amd") or "at::native" in row["Kernel_Name"]:
                continue
            ms[k].append(round((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6, 3))
            scratch[k] = int(row["Scratch_Size"])
            vgpr[k] = int(row["VGPR_Count"]) + int(row.get("Accum_VGPR_Count") or 0)
            lds[k] = int(row["LDS_Block_Size"])
    json.dump({"source": f"rocprofv3 --kernel-trace ({tag_dir})",
               "dispatches_ms": ms, "scratch_bytes_per_lane": scratch, "vgprs": vgpr,
               "lds_bytes_per_workgroup": lds}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
