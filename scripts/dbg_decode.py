import sys, os
sys.path.insert(0, 'tests'); sys.path.insert(0, 'oracle')
from conftest import load_product
import oracle as O
from cases import small_cases
dg = load_product(); o = O.Oracle(); ctx = dg.Context(0)
for name, R, V, p, q in small_cases()[:24]:
    d = o.encode(1, R, V, p=p, q=q)
    try:
        out = dg.decode(R, d, ignore_hash=True, ctx=ctx)
    except Exception as e:
        print(name, "EXC", e); continue
    if out == V:
        print(name, "ok"); continue
    diffs = [i for i in range(min(len(out), len(V))) if out[i] != V[i]]
    print(name, "len", len(out), len(V), "ndiff", len(diffs), "first", diffs[:5])
    cmds = o.diff_onepass(R, V, p, q)
    if diffs:
        f = diffs[0]
        for c in cmds:
            vo = c[1]; ln = c[-1]
            if vo <= f < vo + ln: print("   at cmd", c, "index", cmds.index(c)); break
    print("   out", out[diffs[0]:diffs[0]+16] if diffs else b"", "exp", V[diffs[0]:diffs[0]+16] if diffs else b"")
