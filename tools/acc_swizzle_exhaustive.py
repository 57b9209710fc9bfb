"""Exhaustive GF(2)-linear search of the v4 accumulator swizzle (see acc_swizzle_search.py).
slot = ((z&3)*4 + pg*2 + h) ^ f(z>>2), f linear 6->4 bits.  A phase is conflict-free when
the slot deltas of the lane-group's free variables are linearly independent."""
import numpy as np
Q, T = 4, 4
# z-bit deltas (as ints) of each free variable, per phase.  line bits: ll0=1, ll1=2, ll2=4.
# read groups: free pg, j0, j1, ll0 with ll2 = ll0 ^ j1 ^ c  -> j1, ll0 also toggle ll2
# write groups: free pg, j0, ll2
def zdelta_line(bitmask, Y):
    # z bits of line bits for section Y (line bit b -> z bit)
    if Y == 0: pos = [0, 1, 2, 3, 4, 5]
    elif Y == 1: pos = [0, 1, 2, 3, 6, 7]
    elif Y == 2: pos = [0, 1, 4, 5, 6, 7]
    else: pos = [2, 3, 4, 5, 6, 7]
    r = 0
    for b in range(6):
        if bitmask >> b & 1: r |= 1 << pos[b]
    return r
def jbits(Y):
    return {0: (6, 7), 1: (4, 5), 2: (2, 3), 3: (0, 1)}[Y]
phases = []
for Y in range(4):   # 3 = finish (j' = j or j + k: still a bijection of j, delta same for j0 when x = j^... use j)
    j0, j1 = (1 << jbits(Y)[0]), (1 << jbits(Y)[1])
    ll0, ll2 = zdelta_line(1, Y), zdelta_line(4, Y)
    phases.append(("r", [("pg", 0), ("z", j0), ("z", j1 ^ ll2), ("z", ll0 ^ ll2)]))
    if Y < 3:
        phases.append(("w", [("pg", 0), ("z", j0), ("z", ll2)]))
def slot_delta(kind, z, F):
    # base part: (z&3)*4 (+pg*2); f part from z>>2
    if kind == "pg":
        return np.full(F.shape[1], 2, dtype=np.int64)
    base = (z & 3) * 4
    hi = z >> 2
    out = np.zeros(F.shape[1], dtype=np.int64)
    for o in range(4):
        par = np.zeros(F.shape[1], dtype=np.int64)
        for b in range(6):
            if hi >> b & 1: par ^= (F[o] >> b) & 1
        out |= par << o
    return out ^ base
def rank_ok(vecs, bits):
    # Gaussian elimination over GF(2), vectorised over candidates
    mask = (1 << bits) - 1
    vs = [v & mask for v in vecs]
    ok = np.ones(vs[0].shape, bool)
    basis = []
    for v in vs:
        r = v.copy()
        for bv, piv in basis:
            r = np.where((r >> piv) & 1 == 1, r ^ bv, r)
        piv = np.zeros_like(r)
        nz = r != 0
        ok &= nz
        # pivot = lowest set bit
        low = r & -r
        piv = np.log2(np.maximum(low, 1)).astype(np.int64)
        basis.append((r, piv))
    return ok
N = 1 << 24
sols = []
for start in range(0, N, 1 << 20):
    c = np.arange(start, start + (1 << 20), dtype=np.int64)
    F = np.stack([(c >> (6 * o)) & 63 for o in range(4)])
    ok = np.ones(c.shape, bool)
    for kind, vars_ in phases:
        vecs = [slot_delta(k, z, F) for k, z in vars_]
        ok &= rank_ok(vecs, 4 if kind == "r" else 3)
    idx = np.nonzero(ok)[0]
    if len(idx):
        sols.extend((c[idx][:5]).tolist())
        break
print("solutions:", [[hex((s >> (6 * o)) & 63) for o in range(4)] for s in sols])
