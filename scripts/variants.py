#!/usr/bin/env python3
"""Build A/B variants of libgwaoi.so (compile-time knobs) under variants/, for scripts/variants_run.sh.

usage: python scripts/variants.py name=DEF1,DEF2[:bench args] name2=... ; a name with no defines is the
default build; text after ':' is passed to bench.py for that variant (e.g. ":--cells-per-dist 5").
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from goworld_amd import build  # noqa: E402

os.makedirs(os.path.join(ROOT, "variants"), exist_ok=True)
names = []
for arg in sys.argv[1:]:
    name, _, rest = arg.partition("=")
    defs, _, bargs = rest.partition(":")
    out = os.path.join(ROOT, "variants", f"libgwaoi_{name}.so")
    build.build(force=True, out=out, defines=[d for d in defs.split(",") if d])
    with open(os.path.join(ROOT, "variants", f"args_{name}"), "w") as f:
        f.write(bargs + "\n")
    names.append(name)
with open(os.path.join(ROOT, "variants", "LIST"), "w") as f:
    f.write(" ".join(names) + "\n")
print("built", names)
