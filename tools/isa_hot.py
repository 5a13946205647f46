"""Largest loop of one kernel in a hipcc -S listing: instruction classes of its body and the
(previous instruction, s_nop, next instruction) contexts of its s_nop pads (development tool).
usage: python tools/isa_hot.py kernels.s KERNEL_SYMBOL"""
import collections
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from isa_loops import klass  # noqa: E402

L = open(sys.argv[1]).read().split("\n")
fn = sys.argv[2]
s = next(i for i, l in enumerate(L) if l.startswith(fn + ":"))
e = next(i for i in range(s, len(L)) if L[i].startswith(".Lfunc_end"))
labels = {}
best = None
for i in range(s, e):
    m = re.match(r"^(\.LBB\d+_\d+):", L[i])
    if m:
        labels[m.group(1)] = i
    m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", L[i])
    if m and m.group(2) in labels and (best is None or i - labels[m.group(2)] > best[1] - best[0]):
        best = (labels[m.group(2)], i)
a, b = best
ins = []
for i in range(a, b + 1):
    t = L[i].strip()
    if t and not t.startswith(";") and not t.startswith(".") and not t.endswith(":"):
        ins.append(t)
cls = collections.Counter()
for t in ins:
    op = t.split()[0]
    cls["s_nop" if op == "s_nop" else klass(op)] += 1
print(f"loop {L[a].split(':')[0]} lines {a}-{b}: {len(ins)} instructions, "
      f"VALU {sum(1 for t in ins if t.startswith('v_'))}, s_nop {cls['s_nop']}")
for k, v in cls.most_common():
    print(f"  {v:6d}  {k}")
ctx = collections.Counter()
for j, t in enumerate(ins):
    if t.startswith("s_nop"):
        p = next(x for x in reversed(ins[:j]) if not x.startswith("s_nop")).split()[0]
        n = next(x for x in ins[j + 1:] if not x.startswith("s_nop")).split()[0]
        ctx[(p, t, n)] += 1
print("s_nop contexts:")
for k, v in ctx.most_common(12):
    print(f"  {v:6d}  {k}")
