"""Per-kernel mean of every PMC counter in rocprofv3 --pmc CSV outputs, plus
derived utilisation figures for the SQ passes of tools/profile_round.sh.

    python tools/pmc_summary.py gpurun_out/<tag> > profiles/r01/pmc_sq_<name>.json

Derived (per kernel, means over dispatches):
  lane_util      = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU)  active lanes per VALU issue cycle
  valu_issue     = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES                 VALU-busy fraction of a wave's life
  fp64_valu_ops  = FMA_F64 + MUL_F64 + ADD_F64 + TRANS_F64 (wave instructions)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    s = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return s.split("(")[0].split("::")[-1]


def load(d):
    acc = defaultdict(lambda: defaultdict(float))   # (kernel, dispatch) -> counter -> sum over XCD rows
    for path in glob.glob(os.path.join(d, "pmc_*", "*counter_collection.csv")):
        with open(path) as f:
            for row in csv.DictReader(f):
                acc[(short(row["Kernel_Name"]), path, row["Dispatch_Id"])][row["Counter_Name"]] += float(
                    row["Counter_Value"])
    per = defaultdict(lambda: defaultdict(list))
    for (k, _, _), cs in acc.items():
        for c, v in cs.items():
            per[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}


def main(d):
    res = {"source": d, "units": "per dispatch (mean); SQ counters summed over XCDs"}
    for k, cs in sorted(load(d).items()):
        if k.startswith("__amd") or "elementwise" in k:
            continue
        out = dict(cs)
        if cs.get("SQ_ACTIVE_INST_VALU"):
            if "SQ_THREAD_CYCLES_VALU" in cs:
                out["lane_util"] = cs["SQ_THREAD_CYCLES_VALU"] / (64.0 * cs["SQ_ACTIVE_INST_VALU"])
            if cs.get("SQ_WAVE_CYCLES"):
                out["valu_issue"] = cs["SQ_ACTIVE_INST_VALU"] / cs["SQ_WAVE_CYCLES"]
        f64 = [cs.get(c) for c in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                   "SQ_INSTS_VALU_TRANS_F64")]
        if all(v is not None for v in f64):
            out["fp64_valu_ops"] = sum(f64)
        res[k] = out
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
