"""Summarise a rocprofv3 rocpd SQLite database: per kernel, dispatches,
mean duration and the mean of each PMC counter per dispatch.

    python tools/rocpd_pmc.py gpurun_out/pmc1/pmc1_results.db
"""
import sqlite3
import sys
from collections import defaultdict


def tables(cur):
    return {r[0].rsplit("_", 5)[0] if r[0].count("_") > 5 else r[0]: r[0]
            for r in cur.execute("select name from sqlite_master where type='table'")}


def main(path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    names = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    T = lambda p: next(n for n in names if n.startswith(p))  # noqa: E731
    ks = T("rocpd_info_kernel_symbol")
    kd = T("rocpd_kernel_dispatch")
    cols = [r[1] for r in cur.execute(f"pragma table_info({ks})")]
    namecol = "kernel_name" if "kernel_name" in cols else ("display_name" if "display_name" in cols else cols[1])
    sym = {r[0]: r[1] for r in cur.execute(f"select id, {namecol} from {ks}")}
    kcols = [r[1] for r in cur.execute(f"pragma table_info({kd})")]
    disp = {}
    for r in cur.execute(f"select id, kernel_id, start, end, event_id from {kd}"):
        disp[r[4]] = (sym.get(r[1], str(r[1])), r[3] - r[2])
    dur = defaultdict(list)
    for k, d in disp.values():
        dur[k].append(d)
    pe = T("rocpd_pmc_event")
    pi = T("rocpd_info_pmc")
    pcols = [r[1] for r in cur.execute(f"pragma table_info({pi})")]
    pname = {r[0]: r[1] for r in cur.execute(f"select id, name from {pi}")}
    vals = defaultdict(lambda: defaultdict(float))
    for ev, pmc, v in cur.execute(f"select event_id, pmc_id, value from {pe}"):
        if ev in disp:
            vals[disp[ev][0]][pname.get(pmc, pmc)] += v
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        n = len(dur[k])
        short = k.split("(")[0][-60:]
        print(f"{short}: {n} dispatches, mean {sum(dur[k]) / n / 1e6:.3f} ms")
        for c, v in sorted(vals[k].items()):
            print(f"    {c:28s} {v / n:.6g}")


if __name__ == "__main__":
    main(sys.argv[1])
