"""numpy restatement of the streaming decodes' algebra (test infrastructure, CPU only).

The HIP kernels k_stream_local (stream_local.hpp), k_stream_local256 (stream_local256.hpp) and
k_stream_fused2 (stream_fused2.hpp, stream_decode.hpp) decode q = 4, t = 4 codes in the syndrome form of the
reference's layered decode (decode.rs:167-408): per layer the RS reconstruct is the unique
codeword through the first k+nu present shards, so the erased U values are H_K^-1 S with
S = sum over used nodes of H_i U_i.  This module replays the kernels' step order on whole
sub-chunks with numpy (no GPU) so the CPU suite checks the algebra -- level order, dropped
companion terms, the in-lane / g2-line / pair-inversion steps of the local kernel and the
per-level rounds of the fused kernel -- against the oracle for every eligible erasure pattern.
The kernels themselves are checked on the GPU (tests/test_gpu_stream_local.py,
tests/test_gpu_stream_decode.py)."""
import numpy as np

POLY = 0x11D
GAMMA = 2


def _gf_tables():
    exp = np.zeros(512, dtype=np.int64)
    log = np.zeros(256, dtype=np.int64)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= POLY
    exp[255:510] = exp[0:255]
    mul = np.zeros((256, 256), dtype=np.uint8)
    for a in range(1, 256):
        mul[a, 1:] = exp[log[a] + log[np.arange(1, 256)]]
    return mul, exp, log


MUL, EXP, LOG = _gf_tables()


def gmul(c, v):
    """GF(2^8) constant c times the byte array v."""
    return MUL[int(c)][v]


def ginv(a):
    return int(EXP[255 - LOG[a]])


def gf_invert(m):
    """Inverse of a small GF(2^8) matrix (Gauss-Jordan)."""
    n = len(m)
    a = [list(map(int, r)) + [1 if i == j else 0 for j in range(n)] for i, r in enumerate(m)]
    for c in range(n):
        p = next(r for r in range(c, n) if a[r][c])
        a[c], a[p] = a[p], a[c]
        iv = ginv(a[c][c])
        a[c] = [int(MUL[iv][x]) for x in a[c]]
        for r in range(n):
            if r != c and a[r][c]:
                f = a[r][c]
                a[r] = [x ^ int(MUL[f][y]) for x, y in zip(a[r], a[c])]
    return [r[n:] for r in a]


class Code:
    """(k, m, d) with q = m = 4, t = 4: internal nodes 0..15 (data, nu shortened zero nodes,
    parity), H = [G | I] from the oracle's RS matrix."""

    def __init__(self, oracle_mod, k, m=4):
        self.k, self.m, self.q, self.t = k, m, 4, 4
        self.nu = 16 - k - m
        self.K = k + self.nu
        rs = oracle_mod.rs_matrix(self.K, m)  # (K + m) x K, the first K rows the identity
        self.H = np.zeros((4, 16), dtype=np.int64)
        for p in range(4):
            for i in range(self.K):
                self.H[p, i] = int(rs[self.K + p, i])
            self.H[p, self.K + p] = 1
        self.n = k + m

    def internal(self, e):
        return e if e < self.k else e + self.nu

    @staticmethod
    def digit(z, y):
        return (z >> (2 * (3 - y))) & 3

    @staticmethod
    def with_digit(z, y, x):
        sh = 2 * (3 - y)
        return (z & ~(3 << sh)) | (x << sh)


def _setup(code, chunks, erased_ext):
    """Internal chunk images C[i] (256 x sc), erased set, used set, K, the rows of H_K^-1 of the
    erased nodes (r order: ascending internal index, as the host) and the A_i tables."""
    sc = chunks.shape[1] // 256
    E = sorted(code.internal(e) for e in erased_ext)
    C = np.zeros((16, 256, sc), dtype=np.uint8)
    for e in range(code.n):
        i = code.internal(e)
        if i not in E:
            C[i] = chunks[e].reshape(256, sc)
    used, Kset = [], []
    for i in range(16):
        if i not in E and len(used) < code.K:
            used.append(i)
        else:
            Kset.append(i)
    hinv = gf_invert([[code.H[p, i] for i in Kset] for p in range(4)])
    rows = [hinv[Kset.index(e)] for e in E]  # row of H_K^-1 per erased r
    A = {}
    for i in range(16):  # A_i[r] = (H_K^-1 gamma H_i)[e_r]
        A[i] = [0] * len(E)
        for r in range(len(E)):
            v = 0
            for j in range(4):
                v ^= int(MUL[rows[r][j]][MUL[GAMMA][code.H[j, i]]])
            A[i][r] = v
    return C, E, set(used), rows, A


def _syndromes_presolved(code, C, E, used, rows):
    """Phase A + presolve: V_r(z) = row e_r of H_K^-1 S(z), S with the terms gamma C(e, z') of
    erased companions dropped and the Out terms of erased nodes with present companions folded in
    (so V is C of every layer whose dropped terms are zero)."""
    Eset = set(E)
    sc = C.shape[2]
    V = np.zeros((len(E), 256, sc), dtype=np.uint8)
    for z in range(256):
        S = np.zeros((4, sc), dtype=np.uint8)
        for i in range(16):
            y, x = divmod(i, 4)
            zy = code.digit(z, y)
            comp = 4 * y + zy
            zs = code.with_digit(z, y, x)
            if i in used:
                u = C[i, z].copy()
                if zy != x and comp not in Eset:
                    u ^= gmul(GAMMA, C[comp, zs])
            elif i in Eset and zy != x and comp not in Eset:
                u = gmul(GAMMA, C[comp, zs])  # Out(e, z): recover_type1_erasure
            else:
                continue
            for p in range(4):
                S[p] ^= gmul(code.H[p, i], u)
        for r in range(len(E)):
            for j in range(4):
                V[r, z] ^= gmul(rows[r][j], S[j])
    return V


def presolved_by_source(code, C, E, used, rows, A, G):
    """k_stream_local256's phase A (stream_local256.hpp) for one or two erased nodes in section G: per
    group b (digit G = b) S_b takes the sections != G as above and only the OWN terms H_i C(i, z)
    of section G; the coupled terms gamma H_(G,b) C((G, X), z[G := b]) of section G are collected
    by source -- node (G, X) at group b != X adds A_(G,b)[r] C((G, X), z') to row r at z'[G := X]
    when (G, b) is used or erased (its Out term).  Equals _syndromes_presolved."""
    Eset = set(E)
    sc = C.shape[2]
    V = np.zeros((len(E), 256, sc), dtype=np.uint8)
    for z in range(256):
        S = np.zeros((4, sc), dtype=np.uint8)
        for i in range(16):
            y, x = divmod(i, 4)
            zy = code.digit(z, y)
            comp = 4 * y + zy
            zs = code.with_digit(z, y, x)
            if y == G:
                if i in used:
                    u = C[i, z]
                else:
                    continue
            elif i in used:
                u = C[i, z].copy()
                if zy != x and comp not in Eset:
                    u ^= gmul(GAMMA, C[comp, zs])
            elif i in Eset and zy != x and comp not in Eset:
                u = gmul(GAMMA, C[comp, zs])
            else:
                continue
            for p in range(4):
                S[p] ^= gmul(code.H[p, i], u)
        for r in range(len(E)):
            for j in range(4):
                V[r, z] ^= gmul(rows[r][j], S[j])
        b = code.digit(z, G)
        if (4 * G + b) in used or (4 * G + b) in Eset:
            for X in range(4):
                src = 4 * G + X
                if X == b or src in Eset:
                    continue  # the red node; an erased source has no data (dropped, solve step ii)
                zt = code.with_digit(z, G, X)
                for r in range(len(E)):
                    V[r, zt] ^= gmul(A[4 * G + b][r], C[src, z])
    return V


def local_eligible(code, erased_ext):
    per = [0] * 4
    for e in erased_ext:
        per[code.internal(e) // 4] += 1
    nz = sorted([p for p in per if p], reverse=True)
    return 1 <= len(erased_ext) <= 4 and len(nz) <= 2 and (len(nz) < 2 or nz[1] == 1)


def local_decode(code, chunks, erased_ext):
    """k_stream_local's steps: presolve, (i) g2-line terms of the slots outside E_G, (ii) in-lane
    terms of the slots in E_G, (iii) g2-line terms of the slots in E_G, (iv) both-erased pairs.
    Returns {internal erased node: 256 x sc C}."""
    C, E, used, rows, A = _setup(code, chunks, erased_ext)
    per = [0] * 4
    for i in E:
        per[i // 4] += 1
    G = max(range(4), key=lambda y: (per[y], -y))
    g2 = next((y for y in range(4) if y != G and per[y]), -1)
    EG = [i % 4 for i in E if i // 4 == G]
    rix = {e: r for r, e in enumerate(E)}
    V = _syndromes_presolved(code, C, E, used, rows)
    ne = len(E)

    def line_g2(slots):
        x2 = next(i % 4 for i in E if i // 4 == g2)
        r2 = rix[4 * g2 + x2]
        for z in range(256):
            if code.digit(z, G) not in slots or code.digit(z, g2) != x2:
                continue
            for X in range(4):
                if X == x2 or (4 * g2 + X) not in used:
                    continue
                src = V[r2, code.with_digit(z, g2, X)]
                for r in range(ne):
                    V[r, z] ^= gmul(A[4 * g2 + X][r], src)

    if g2 >= 0:
        line_g2([g for g in range(4) if g not in EG])  # (i)
    for z in range(256):  # (ii)
        g = code.digit(z, G)
        if g not in EG:
            continue
        rg = rix[4 * G + g]
        for Aa in range(4):
            if Aa in EG or (4 * G + Aa) not in used:
                continue
            src = V[rg, code.with_digit(z, G, Aa)]
            for r in range(ne):
                V[r, z] ^= gmul(A[4 * G + Aa][r], src)
    if g2 >= 0:
        line_g2(EG)  # (iii)
    dinv = ginv(1 ^ int(MUL[GAMMA][GAMMA]))
    for g in EG:  # (iv)
        for x in EG:
            if x <= g:
                continue
            rx, rg = rix[4 * G + x], rix[4 * G + g]
            for z in range(256):
                if code.digit(z, G) != g:
                    continue
                zx = code.with_digit(z, G, x)
                u1, u2 = V[rx, z].copy(), V[rg, zx].copy()
                V[rx, z] = gmul(dinv, u1 ^ gmul(GAMMA, u2))
                V[rg, zx] = gmul(dinv, u2 ^ gmul(GAMMA, u1))
    return {e: V[rix[e]] for e in E}


def fused_decode(code, chunks, erased_ext):
    """k_stream_fused2's rounds (one erasure per y-section): presolve, then per iscore
    level L >= 1 every layer of level L adds sum over its red sections Y and used X != x_e(Y) of
    A_(Y,X) C(e_Y, z[Y := X]) -- sources of level L - 1, final before the round."""
    C, E, used, rows, A = _setup(code, chunks, erased_ext)
    rix = {e: r for r, e in enumerate(E)}
    xe = {i // 4: i % 4 for i in E}
    V = _syndromes_presolved(code, C, E, used, rows)

    def level(z):
        return sum(1 for y, x in xe.items() if code.digit(z, y) == x)

    for L in range(1, 5):
        for z in [z for z in range(256) if level(z) == L]:
            for Y, x in xe.items():
                if code.digit(z, Y) != x:
                    continue
                for X in range(4):
                    if X == x or (4 * Y + X) not in used:
                        continue
                    src = V[rix[4 * Y + x], code.with_digit(z, Y, X)]
                    for r in range(len(E)):
                        V[r, z] ^= gmul(A[4 * Y + X][r], src)
    return {e: V[rix[e]] for e in E}
