"""Where a kernel waits on vector memory: every s_waitcnt with a vmcnt in a kernel of a `-g` device assembly,
mapped to its source line and followed by the first instructions it guards (the registers whose pending write forces
the wait).  A vmcnt(0) inside a loop that prefetches (loads issued one iteration ahead) usually means a rare path left
a load outstanding into registers the common path reuses.
    hipcc --offload-arch=gfx950 -O3 -g --cuda-device-only -S -o k.s <src> [flags]
    python scripts/waitcnt_map.py k.s <kernel-name-substring> [first_line last_line]"""
import re
import sys

path, name = sys.argv[1], sys.argv[2]
lo, hi = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (0, 1 << 30)
text = open(path).read().split("\n")
start = next(i for i, l in enumerate(text) if re.match(r"^_Z\S*" + re.escape(name) + r"\S*:", l))
loc = None
for i in range(start, len(text)):
    l = text[i]
    if "s_endpgm" in l:
        break
    m = re.match(r"\s*\.loc\s+\d+\s+(\d+)\s+(\d+)", l)
    if m:
        loc = (int(m.group(1)), int(m.group(2)))
    if re.search(r"s_waitcnt.*vmcnt", l) and loc and lo <= loc[0] <= hi:
        nxt = [x.strip() for x in text[i + 1:i + 8] if x.strip() and not x.strip().startswith((".loc", ";", ".Ltmp"))]
        print(f"{loc[0]}:{loc[1]}  {l.strip():32s} | {' ; '.join(nxt[:2])}")
