"""Liveness of the staged planner's U workspace slots: how many U values (per byte position)
are live at once if the whole plan runs per tile in op order, and how many distinct
inputs/outputs it touches.  Decides whether a fused single-launch executor fits in LDS."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import plan_emu as E
from clay_amd import ClayCode

def analyse(name, c, kind, mask=None, want=None, lost=0):
    tn = c.q * c.t
    ops, srcs, stages = E.export_plan(c, kind, mask, want, lost)
    first, last = {}, {}
    n_in = set(); n_out = 0; nsrc = 0
    for i, (dst_base, dst_slot, sb, ns) in enumerate(ops):
        for j in range(sb, sb + ns):
            b, sl, coef, _ = srcs[j]
            nsrc += 1
            if b == 2 * tn:
                last[sl] = i
            else:
                n_in.add((b, sl))
        if dst_base == 2 * tn:
            first.setdefault(dst_slot, i)
            last.setdefault(dst_slot, i)
        else:
            n_out += 1
    ev = []
    for s in first:
        ev.append((first[s], 1)); ev.append((last[s] + 1, -1))
    ev.sort()
    live = mx = 0
    for _, d in ev:
        live += d; mx = max(mx, live)
    print(f"{name}: ops {len(ops)} levels {len(stages)-1} src terms {nsrc} | U slots {len(first)} max live {mx} "
          f"| distinct input sub-chunks {len(n_in)} outputs {n_out}")

c = ClayCode(10, 4, 13)
tn = 16
m = [0] * tn
for i in (0, 4, 8, 14): m[i] = 1
analyse("decode (10,4,13) {0,4,8,12}", c, 1, m, m)
m = [0] * tn; m[0] = 1
analyse("decode (10,4,13) {0}", c, 1, m, m)
analyse("encode (10,4,13)", c, 0)
c = ClayCode(9, 3, 11)
info = c.minimum_to_repair(0, list(range(1, 12)))
hm = [0] * 12
for h, _ in info: hm[h] = 1
analyse("repair (9,3,11) node 0", c, 2, hm, None, 0)
c = ClayCode(4, 2, 5)
m = [0] * 6; m[0] = 1
analyse("decode (4,2,5) {0}", c, 1, m, m)
