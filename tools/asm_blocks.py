"""Instruction mix per basic block of one kernel in a hipcc -S listing (VALU / SALU / MFMA /
LDS / global / branch), to see where a kernel's instructions go.
Usage: python tools/asm_blocks.py listing.s kernel_symbol [min_valu]"""
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
minv = int(sys.argv[3]) if len(sys.argv) > 3 else 0
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
blocks, cur, name = [], None, "entry"
cnt = dict(v=0, s=0, m=0, l=0, g=0, b=0)
def flush():
    blocks.append((name, dict(cnt)))
for l in lines[start + 1:]:
    if l.startswith(".Lfunc_end"):
        break
    m = re.match(r"^(\.LBB\w+):(.*)", l)
    if m:
        flush()
        name = m.group(1) + (" loop" if "Loop Header" in m.group(2) else "")
        cnt = dict(v=0, s=0, m=0, l=0, g=0, b=0)
        continue
    t = l.strip().split(" ")[0].split("\t")[0]
    if not t or t.startswith((";", ".")):
        continue
    if t.startswith("v_mfma"):
        cnt["m"] += 1
    elif t.startswith("v_"):
        cnt["v"] += 1
    elif t.startswith("s_cbranch") or t.startswith("s_branch"):
        cnt["b"] += 1
    elif t.startswith("s_"):
        cnt["s"] += 1
    elif t.startswith("ds_"):
        cnt["l"] += 1
    elif t.startswith(("global_", "buffer_", "flat_", "scratch_")):
        cnt["g"] += 1
flush()
tot = dict(v=0, s=0, m=0, l=0, g=0, b=0)
for nm, c in blocks:
    for k in tot:
        tot[k] += c[k]
    if c["v"] >= minv:
        print(f"{nm:28s} valu {c['v']:5d} salu {c['s']:4d} mfma {c['m']:3d} lds {c['l']:3d} glob {c['g']:3d} br {c['b']:2d}")
print("total", tot, "blocks", len(blocks))
