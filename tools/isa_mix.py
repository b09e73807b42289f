"""Static instruction mix per function of a hipcc -S (gfx950) assembly file.

    hipcc --offload-arch=gfx950 -O3 ... --offload-device-only -S -o out.s src.hip
    python tools/isa_mix.py out.s [substring]
"""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read().split("\n")
want = sys.argv[2] if len(sys.argv) > 2 else ""
funcs, cur = {}, None
for line in src:
    m = re.match(r"^([.\w]+):\s*; @", line)
    if m:
        cur = m.group(1)
        funcs[cur] = []
        continue
    if cur and line.startswith(".Lfunc_end"):
        cur = None
        continue
    if cur and line.startswith("\t") and not line.strip().startswith((".", ";")):
        funcs[cur].append(line.strip().split()[0])
for name, ins in sorted(funcs.items(), key=lambda kv: -len(kv[1])):
    if want not in name or len(ins) < 50:
        continue
    c = Counter(ins)
    cats = Counter()
    for k, v in c.items():
        cats[k.split("_")[0]] += v
    print(f"{name[:90]}: {len(ins)} instrs  {dict(cats.most_common(8))}")
    print("   ", c.most_common(18))
