"""Per-kernel register and memory resources of the gfx950 code object, from the
device assembly the compiler emits (hipcc --cuda-device-only -S):
arch VGPRs, AccVGPRs, SGPRs, scratch bytes per lane, static LDS, and the
waves/SIMD the register file allows (512 registers per SIMD lane on CDNA4,
shared by arch and acc VGPRs, allocated in granules of 8).

    hipcc --offload-arch=gfx950 <Makefile FLAGS> --cuda-device-only -S -o /tmp/render.s csrc/render.hip
    python tools/kernel_resources.py /tmp/render.s [name-filter ...] > profiles/r03/kernel_resources.json
"""
import json
import re
import sys


def demangle_short(sym):
    m = re.search(r"_GLOBAL__N_1\d+(k_\w+?)(I.*?)?E?Ev", sym) or re.search(r"(k_\w+)", sym)
    name = m.group(1) if m else sym
    targs = re.findall(r"L([ib])(\d+)E", sym[:200])
    if targs:
        name += "<" + ", ".join(("true" if v == "1" else "false") if t == "b" else v for t, v in targs) + ">"
    return name


_cache = {}


def resolve(txt, name):
    """Value of `.set name, expr`, where expr may be max(...) over numbers and
    other symbols (kernels that call out-of-line device functions)."""
    if name in _cache:
        return _cache[name]
    m = re.search(r"^\s+\.set " + re.escape(name) + r", (.+)$", txt, re.M)
    val = 0
    if m:
        expr = m.group(1)
        nums = [int(x) for x in re.findall(r"(?<![\w.])(\d+)(?![\w.])", expr)]
        refs = re.findall(r"([A-Za-z_.$][\w.$]*\.(?:num_vgpr|num_agpr|numbered_sgpr))", expr)
        vals = nums + [resolve(txt, r) for r in refs if r != name]
        val = max(vals) if vals else 0
    _cache[name] = val
    return val


def main():
    path = sys.argv[1]
    filt = sys.argv[2:]
    txt = open(path).read()
    out = {}
    for m in re.finditer(r"^\s+\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", txt, re.M | re.S):
        sym, body = m.group(1), m.group(2)
        name = demangle_short(sym)
        if filt and not any(f in name for f in filt):
            continue
        def field(k):
            f = re.search(r"\.amdhsa_" + k + r"\s+(\S+)", body)
            return f.group(1) if f else None
        vg = resolve(txt, sym + ".num_vgpr")
        ag = resolve(txt, sym + ".num_agpr")
        total = ((vg + 7) // 8) * 8 + ((ag + 7) // 8) * 8 if ag else vg
        out[name] = {
            "arch_vgpr": vg, "acc_vgpr": ag, "sgpr": resolve(txt, sym + ".numbered_sgpr"),
            "scratch_bytes_per_lane": int(field("private_segment_fixed_size") or 0),
            "lds_static_bytes": int(field("group_segment_fixed_size") or 0),
            "waves_per_simd_by_registers": min(8, 512 // max(total, 1)) if total else 8,
        }
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
