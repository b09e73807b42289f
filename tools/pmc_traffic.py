"""HBM traffic per kernel instantiation and per pipeline stage, from rocprofv3
--pmc FETCH_SIZE / WRITE_SIZE CSVs (separate passes, as
/opt/skills/guides/MI355X_MICROARCH.md prescribes).

FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters, TCC EA
requests). gfx950 correction from the guide: FETCH_SIZE reports half of the
bytes of wide coalesced 16-B/lane reads (TCC_EA0_RDREQ x 64 B for 128-B
requests); it is applied here to the read side, which makes the read figure
an upper bound for narrower accesses. WRITE_SIZE is taken as is.

Keys:
  "kernels": per full instantiation (template arguments kept, e.g.
             k_chain_ci<1, 0, false, 0> and k_chain_ci<4, 0, false, 0> apart):
             dispatches, bytes per dispatch (mean), bytes per frame;
  "stages":  per kernel family (k_chain_ci, k_paths_ci, k_film, ...): the SUM
             over its instantiations' dispatches per frame -- a frame's chain
             stage is two concurrent launches at N=1, so the stage's bytes are
             what bench.py's `traffic` reports against the stage's time.
Frames end at each k_merge_film dispatch; frame 0 (the cold frame of a fresh
context) is listed but left out of the stage means.

    python tools/pmc_traffic.py gpurun_out/<tag> > profiles/pmc_readme_1920x1080_s8x8.json
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict


def names(kernel_name):
    """(instantiation, family) of a rocprofv3 kernel name."""
    s = kernel_name.replace("void ", "").replace("(anonymous namespace)::", "").replace("pbrtk::", "")
    s = s.split("(")[0].strip()
    s = re.sub(r"\s+", " ", s)
    fam = s.split("<")[0].split("::")[-1]
    return s, fam


def per_dispatch(path, counter):
    acc = defaultdict(float)
    inst = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            key = row["Dispatch_Id"]
            acc[key] += float(row["Counter_Value"])
            inst[key] = names(row["Kernel_Name"])
    return acc, inst


def main(d):
    fetch, fi = per_dispatch(os.path.join(d, "pmc_fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write, wi = per_dispatch(os.path.join(d, "pmc_write", "write_counter_collection.csv"), "WRITE_SIZE")
    build = None   # the library build the passes ran: profile_round.sh's bench.json of the same directory
    try:
        with open(os.path.join(d, "bench.json")) as f:
            build = json.loads(f.read().strip().splitlines()[-1]).get("build_id")
    except (OSError, ValueError, IndexError):
        pass

    # frame of each dispatch: the k_merge_film dispatches close the frames (in dispatch order)
    inst_all = {**fi, **wi}
    merges = sorted(int(k) for k, v in inst_all.items() if v[1] == "k_merge_film")
    frames = max(len(merges), 1)

    def frame_of(k):
        k = int(k)
        return sum(1 for m in merges if m < k)
    # the cold frame (a fresh context: probe order, no heavy/light split) is frame 0;
    # the stages are the steady-state frames' mean (frames 1..), as the bench times them
    steady = list(range(1, frames)) if frames > 1 else [0]
    kernels = {}
    stage_frames = defaultdict(lambda: defaultdict(lambda: [0.0, 0.0]))
    per_inst = defaultdict(lambda: [[], []])
    for k, (inst, fam) in inst_all.items():
        if fam.startswith("__amd") or "elementwise" in fam:
            continue
        r = fetch.get(k, 0.0) * 2 * 1024.0
        w = write.get(k, 0.0) * 1024.0
        per_inst[inst][0].append(r)
        per_inst[inst][1].append(w)
        f = frame_of(k)
        stage_frames[fam][f][0] += r
        stage_frames[fam][f][1] += w
        kernels.setdefault(inst, {"family": fam})
    for inst, (r, w) in per_inst.items():
        n = len(r)
        kernels[inst].update({"dispatches": n, "read_bytes_per_dispatch": sum(r) / n,
                              "write_bytes_per_dispatch": sum(w) / n,
                              "hbm_bytes_per_dispatch": (sum(r) + sum(w)) / n})
    stages = {}
    for fam, byf in stage_frames.items():
        rs = sum(byf[f][0] for f in steady) / len(steady)
        ws = sum(byf[f][1] for f in steady) / len(steady)
        stages[fam] = {"read_bytes_per_frame": rs, "write_bytes_per_frame": ws, "hbm_bytes_per_frame": rs + ws,
                       "instantiations": sorted(i for i, v in kernels.items() if v["family"] == fam),
                       "per_frame": [byf[f][0] + byf[f][1] for f in range(frames)]}
    res = {"source": d, "build_id": build, "frames": frames, "steady_frames": steady,
           "units": "bytes; per dispatch (mean over the run); stages: per frame, the mean over the "
                    "steady-state frames (1..; frame 0 is the cold frame), per_frame lists every frame",
           "correction": "read = 2 x FETCH_SIZE KiB x 1024 (gfx950 half-count of 128-B requests); "
                         "write = WRITE_SIZE KiB x 1024",
           "kernels": kernels, "stages": dict(stages)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
