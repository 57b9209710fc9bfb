"""v6 layout search generalised to PARTS = 8 (W = 256, 512 lanes): piece (c, part, d) with
v = c | part << 6 | d << 9 (10 bits)."""
import random
import sys
sys.path.insert(0, "tools")
G128 = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
G128 += [[l + 32 for l in g] for g in G128]
def dig(c, y): return (c >> (2 * (2 - y))) & 3
def setdig(c, y, v): s = 2 * (2 - y); return (c & ~(3 << s)) | (v << s)
def par(v): return bin(v).count("1") & 1
def bank(Bm, Hm, node, c, part, d):
    v = c | (part << 6) | (d << 9)
    return sum((par(v & Bm[o]) ^ par(node & Hm[o])) << o for o in range(4))
MAPS = {"part=l&7": lambda l: (l >> 3, l & 7), "part=(l>>3)&7": lambda l: ((l & 7) | ((l >> 6) << 3), (l >> 3) & 7)}
def cost(lm, Bm, Hm, early):
    c = 0
    for w in range(8):
        for g in G128:
            at = [lm(w * 64 + l) for l in g]
            for Y in range(3):
                for x in range(4):
                    for d in range(2):
                        for kind in (0, 1):
                            if kind == 0 and Y == 2 and x >= 2:
                                continue
                            seen = {}
                            for (cc, part) in at:
                                if kind == 0:
                                    a = (x, cc, part, d)
                                else:
                                    cy = dig(cc, Y)
                                    if Y == 2 and cy >= 2:
                                        continue
                                    a = (cy, setdig(cc, Y, x), part, d)
                                seen.setdefault(bank(Bm, Hm, *a), set()).add(a)
                            if seen:
                                c += max(len(s) for s in seen.values()) - 1
                            if c > early:
                                return c
    return c
rng = random.Random(5)
for name, lm in MAPS.items():
    best = None
    for it in range(4000):
        Bm = [rng.randrange(1 << 10) for _ in range(4)]
        Hm = [rng.randrange(4) for _ in range(4)]
        cst = cost(lm, Bm, Hm, best[0] if best else 10 ** 9)
        if best is None or cst < best[0]:
            best = (cst, Bm, Hm)
            if cst == 0:
                break
    print(name, best[0], [hex(b) for b in best[1]], best[2], flush=True)
