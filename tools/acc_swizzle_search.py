"""Search an XOR swizzle for the v4 accumulator layout of (10,4,13) so that the LDS
read-modify-write of every section and the PFT reads are bank-conflict free.
Lane map: b0=pg b1=j0 b2=ll2 b3=j1 b4=ll0 b5=ll1 (matches ds_read_b128 lane groups)."""
import itertools, random
Q, T, A = 4, 4, 256
def lane_attrs(L):
    pg = L & 1; j = ((L >> 1) & 1) | (((L >> 3) & 1) << 1)
    ll = ((L >> 4) & 1) | (((L >> 5) & 1) << 1) | (((L >> 2) & 1) << 2)
    return pg, j, ll
G128 = [[*range(0,4),*range(12,16),*range(20,28)], [*range(4,12),*range(16,20),*range(28,32)]]
G128 += [[l+32 for l in g] for g in G128]
GW128 = [list(range(8*i, 8*i+8)) for i in range(8)]
def wy(Y): return Q ** (T - 1 - Y)
def zl(line, Y): W = wy(Y); return (line // W) * W * Q + line % W
def addr(z, pg, h, f):
    s = ((z & 3) * 4 + pg * 2 + h) ^ f(z)
    return (z >> 2) * 256 + s * 16
def cost(f):
    c = 0
    for wave in range(8):
        accs = []
        for Y in range(3):
            for h in range(2):
                a = {}
                for L in range(64):
                    pg, j, ll = lane_attrs(L)
                    a[L] = addr(zl(wave*8+ll, Y) + j*wy(Y), pg, h, f)
                accs.append(("rw", a))
        for k in range(4):
            for part in range(2 if k else 1):
                for h in range(2):
                    a = {}
                    for L in range(64):
                        pg, j, ll = lane_attrs(L); z0 = (wave*8+ll)*4; x = j ^ k
                        z = z0 + j if (k == 0 or part == 0) else z0 + x
                        a[L] = addr(z, pg, h, f)
                    accs.append(("r", a))
        for kind, a in accs:
            for g in G128:
                sl = {}
                for L in g: sl.setdefault((a[L] // 16) % 16, set()).add(a[L])
                c += max(len(v) for v in sl.values()) - 1
            if kind == "rw":
                for g in GW128:
                    sl = {}
                    for L in g: sl.setdefault((a[L] // 16) % 8, set()).add(a[L])
                    c += max(len(v) for v in sl.values()) - 1
    return c
def lin(M):
    def f(z):
        r = 0
        for o in range(4):
            if bin(z & M[o]).count("1") & 1: r |= 1 << o
        return r
    return f
print("no swizzle:", cost(lambda z: 0))
best = None
rng = random.Random(1)
for it in range(4000):
    M = [rng.randrange(256) & ~3 for _ in range(4)]   # only bits above the slot's own z bits
    c = cost(lin(M))
    if best is None or c < best[0]:
        best = (c, M); print(it, c, [hex(m) for m in M])
        if c == 0: break
