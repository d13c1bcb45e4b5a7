"""Instruction census of the innermost loops of one kernel in a gfx950 assembly listing (hipcc -S):
    python scripts/loop_census.py file.s kernel-substring [top]
Per loop (header label, depth): VALU (packed / f64 / transcendental split), SALU, LDS, VMEM, waits, branches; the loops
ranked by size.  Blocks are attributed to the innermost loop the compiler's "in Loop: Header=" comment names."""
import re
import sys
from collections import defaultdict

path, pat = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 6
L = open(path).read().split("\n")
starts = [i for i, l in enumerate(L) if re.match(r"^[_A-Za-z][\w.]*:\s*(;.*)?$", l) and pat in l]
if not starts:
    raise SystemExit(f"no kernel label containing {pat!r}")
st = starts[0]
en = next(i for i in range(st, len(L)) if L[i].strip().startswith(".Lfunc_end"))
cur = None
loops = defaultdict(lambda: defaultdict(int))
depth = {}
for l in L[st:en]:
    m = re.match(r"^(\.LBB\w+|; %bb\.\d+):.*?(?:in Loop: Header=(\w+) Depth=(\d+)|Header: Depth=(\d+))?\s*$", l)
    if m:
        lab = m.group(1).lstrip(".").replace("; %bb.", "BB_")
        if m.group(2):
            cur = m.group(2)
            depth[cur] = int(m.group(3))
        else:
            cur = None
        continue
    if "=>" in l and "Loop Header: Depth=" in l:
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    op = t.split()[0]
    if cur is None:
        continue
    c = loops[cur]
    c["total"] += 1
    if op.startswith("v_"):
        c["valu"] += 1
        if op.startswith("v_pk_"):
            c["pk"] += 1
        if "_f64" in op:
            c["f64"] += 1
        if any(k in op for k in ("rcp", "rsq", "sqrt", "exp", "log", "sin", "cos")):
            c["trans"] += 1
        if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
            c["xlane"] += 1
        if op.startswith(("v_mov", "v_accvgpr")):
            c["mov"] += 1
        if op.startswith("v_cndmask"):
            c["cndmask"] += 1
    elif op.startswith("s_waitcnt"):
        c["wait"] += 1
    elif op.startswith(("s_cbranch", "s_branch")):
        c["branch"] += 1
    elif op.startswith("s_"):
        c["salu"] += 1
    elif op.startswith("ds_"):
        c["lds"] += 1
    elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        c["vmem"] += 1
rank = sorted(loops.items(), key=lambda kv: -kv[1]["total"])
for h, c in rank[:top]:
    print(f"{h} depth {depth.get(h)}: " + ", ".join(f"{k} {v}" for k, v in sorted(c.items(), key=lambda kv: -kv[1])))
