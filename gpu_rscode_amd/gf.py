"""Pure-numpy Galois-field oracle, GF(2^w) for w in {4, 8, 16}.

Independent of the C++/HIP code paths; every native result is tested against it.

Parity with the reference:
  * GF(2^8), primitive polynomial 0x11D (``src/matrix.cu:49``, ``src/cpu-rs.c:37``),
  * GF(2^4) poly 0x13 and GF(2^16) poly 0x1100B (``src/galoisfield.cu:22-25``, unbuilt there),
  * the reference's ``gf_pow`` quirk ``pow(0, e) == 1`` (``src/matrix.cu:204-208``) in
    :meth:`GF.pow_ref`, which the reference Vandermonde ``E[i][j] = (j+1)^i`` depends on for k >= 256.
"""
from __future__ import annotations

import itertools
from functools import lru_cache

import numpy as np

POLYS = {4: 0x13, 8: 0x11D, 16: 0x1100B}


class SingularMatrixError(ValueError):
    """Raised when a GF matrix has no inverse (an unrecoverable erasure pattern)."""


class GF:
    """GF(2^w) arithmetic over numpy integer arrays."""

    def __init__(self, w: int = 8, poly: int | None = None):
        if w not in POLYS and poly is None:
            raise ValueError(f"unsupported field width {w}")
        self.w = w
        self.poly = poly if poly is not None else POLYS[w]
        self.order = 1 << w
        self.dtype = np.uint8 if w <= 8 else np.uint16
        n = self.order - 1
        exp = np.zeros(2 * n, dtype=np.int64)
        log = np.full(self.order, -1, dtype=np.int64)
        x = 1
        for i in range(n):
            exp[i] = exp[i + n] = x
            log[x] = i
            x <<= 1
            if x & self.order:
                x ^= self.poly
        if np.any(log[1:] < 0):
            raise ValueError(f"polynomial {self.poly:#x} is not primitive for w={w}")
        self.exp = exp
        self.log = log

    # ---- scalar / elementwise -----------------------------------------------------------------
    def mul(self, a, b):
        a = np.asarray(a, dtype=np.int64)
        b = np.asarray(b, dtype=np.int64)
        r = self.exp[(self.log[a] + self.log[b]) % (self.order - 1)]
        return np.where((a == 0) | (b == 0), 0, r).astype(np.int64)

    def inv(self, a):
        a = np.asarray(a, dtype=np.int64)
        if np.any(a == 0):
            raise ZeroDivisionError("inverse of 0 in GF")
        return self.exp[(self.order - 1 - self.log[a]) % (self.order - 1)]

    def div(self, a, b):
        return self.mul(a, self.inv(b))

    def pow(self, a: int, e: int) -> int:
        if e == 0:
            return 1
        if a == 0:
            return 0
        return int(self.exp[(int(self.log[a]) * e) % (self.order - 1)])

    def pow_ref(self, a: int, e: int) -> int:
        """Reference ``gf_pow``: exp[(log a * e) % 255] with log(0) treated as 510 -> pow(0,e)=1."""
        la = 2 * (self.order - 1) if a == 0 else int(self.log[a])
        return int(self.exp[(la * e) % (self.order - 1)])

    def mul_table(self, c: int) -> np.ndarray:
        """Row ``c * x`` for every x in the field (the map a coefficient applies to a symbol)."""
        return self.mul(c, np.arange(self.order)).astype(self.dtype)

    # ---- matrices -------------------------------------------------------------------------------
    def matmul(self, a: np.ndarray, b: np.ndarray) -> np.ndarray:
        a = np.asarray(a, dtype=np.int64)
        b = np.asarray(b, dtype=np.int64)
        out = np.zeros((a.shape[0], b.shape[1]), dtype=np.int64)
        for t in range(a.shape[1]):
            out ^= self.mul(a[:, t : t + 1], b[t : t + 1, :])
        return out.astype(self.dtype)

    def gemm(self, coeff: np.ndarray, data: np.ndarray) -> np.ndarray:
        """out[i] = XOR_j coeff[i,j] * data[j] for (m x k) coeff and (k x C) symbol rows."""
        coeff = np.asarray(coeff)
        data = np.asarray(data)
        m, k = coeff.shape
        out = np.zeros((m, data.shape[1]), dtype=self.dtype)
        for i in range(m):
            for j in range(k):
                c = int(coeff[i, j])
                if c == 0:
                    continue
                out[i] ^= data[j] if c == 1 else self.mul_table(c)[data[j]]
        return out

    def invert(self, a: np.ndarray) -> np.ndarray:
        """Gauss-Jordan with row pivoting; raises SingularMatrixError."""
        a = np.array(a, dtype=np.int64)
        n = a.shape[0]
        r = np.eye(n, dtype=np.int64)
        for c in range(n):
            nz = np.nonzero(a[c:, c])[0]
            if nz.size == 0:
                raise SingularMatrixError(f"singular matrix (no pivot in column {c})")
            p = c + int(nz[0])
            if p != c:
                a[[c, p]] = a[[p, c]]
                r[[c, p]] = r[[p, c]]
            ip = int(self.inv(a[c, c]))
            a[c] = self.mul(a[c], ip)
            r[c] = self.mul(r[c], ip)
            for row in range(n):
                if row != c and a[row, c]:
                    f = int(a[row, c])
                    a[row] ^= self.mul(f, a[c])
                    r[row] ^= self.mul(f, r[c])
        return r.astype(self.dtype)

    def is_invertible(self, a: np.ndarray) -> bool:
        try:
            self.invert(a)
            return True
        except SingularMatrixError:
            return False

    # ---- coding matrices ------------------------------------------------------------------------
    def vandermonde_ref(self, k: int, p: int) -> np.ndarray:
        """Reference encoding block E[i][j] = (j+1)^i (``src/matrix.cu:752-759``)."""
        return np.array([[self.pow_ref((j + 1) % self.order, i) for j in range(k)] for i in range(p)], dtype=self.dtype)

    def cauchy(self, k: int, p: int) -> np.ndarray:
        """MDS Cauchy block C[i][j] = 1/(x_i + y_j), x_i = k+i, y_j = j."""
        if k + p > self.order:
            raise ValueError("cauchy needs k + p <= field order")
        return np.array([[int(self.inv((k + i) ^ j)) for j in range(k)] for i in range(p)], dtype=self.dtype)

    def sys_vandermonde(self, k: int, p: int) -> np.ndarray:
        """MDS systematic Vandermonde: V[k:] @ inv(V[:k]) with V[r][j] = r^j, r = 0..n-1."""
        n = k + p
        if n > self.order:
            raise ValueError("sys_vandermonde needs k + p <= field order")
        v = np.array([[self.pow(r, j) for j in range(k)] for r in range(n)], dtype=np.int64)
        return self.matmul(v[k:], self.invert(v[:k]))

    def encoding_matrix(self, kind: str, k: int, p: int) -> np.ndarray:
        if kind in ("vandermonde", "vand", "ref"):
            return self.vandermonde_ref(k, p)
        if kind == "cauchy":
            return self.cauchy(k, p)
        if kind in ("sys_vandermonde", "sysvand"):
            return self.sys_vandermonde(k, p)
        raise ValueError(f"unknown matrix kind {kind!r}")

    def generator(self, e: np.ndarray) -> np.ndarray:
        k = e.shape[1]
        return np.vstack([np.eye(k, dtype=self.dtype), e.astype(self.dtype)])

    def decode_matrix(self, g: np.ndarray, rows) -> np.ndarray:
        rows = list(rows)
        return self.invert(np.asarray(g)[rows])

    def singular_patterns(self, g: np.ndarray, k: int):
        """All k-subsets of generator rows that are NOT invertible (SURVEY §2.2 census)."""
        n = g.shape[0]
        return [s for s in itertools.combinations(range(n), k) if not self.is_invertible(np.asarray(g)[list(s)])]


@lru_cache(maxsize=None)
def field(w: int = 8) -> GF:
    return GF(w)


GF256 = field(8)


# ---- GF(2)-linear byte maps (what the gfx950 v_perm kernel applies) ------------------------------
def byte_map_gf256(c: int) -> np.ndarray:
    """x -> c*x over GF(2^8)."""
    return GF256.mul_table(int(c)).astype(np.uint8)


def byte_map_gf16_nibbles(c: int) -> np.ndarray:
    """The design doc's "GF(16) method" (``doc/design.tex:190-209``, tables ``src/gf16.h``): each
    byte is two independent GF(2^4) symbols, both multiplied by c."""
    f = field(4)
    t = f.mul_table(int(c) & 15).astype(np.int64)
    x = np.arange(256)
    return ((t[x >> 4] << 4) | t[x & 15]).astype(np.uint8)


def is_linear(byte_map: np.ndarray) -> bool:
    x = np.arange(256)
    basis = byte_map[1 << np.arange(8)].astype(np.int64)
    pred = np.zeros(256, dtype=np.int64)
    for b in range(8):
        pred ^= np.where((x >> b) & 1, basis[b], 0)
    return bool(np.array_equal(pred, byte_map.astype(np.int64))) and byte_map[0] == 0


def perm_record(byte_map: np.ndarray) -> np.ndarray:
    """8 uint32 words: the v_perm 3-chunk tables of a GF(2)-linear byte map (see
    ``csrc/include/gfrs/gf256.h``): T0[v]=L(v), T1[v]=L(v<<3) (v<8), T2[v]=L(v<<6) (v<4)."""
    bm = np.asarray(byte_map, dtype=np.uint8)
    t0 = bm[np.arange(8)]
    t1 = bm[np.arange(8) << 3]
    t2 = bm[np.arange(4) << 6]
    words = np.zeros(8, dtype=np.uint32)
    words[0:2] = np.frombuffer(t0.tobytes(), dtype="<u4")
    words[2:4] = np.frombuffer(t1.tobytes(), dtype="<u4")
    words[4] = np.frombuffer(t2.tobytes(), dtype="<u4")[0]
    return words


def perm_apply(words: np.ndarray, x: np.ndarray) -> np.ndarray:
    """Host emulation of the device lookup (for tests)."""
    b = np.asarray(words, dtype="<u4").tobytes()
    t0 = np.frombuffer(b[0:8], dtype=np.uint8)
    t1 = np.frombuffer(b[8:16], dtype=np.uint8)
    t2 = np.frombuffer(b[16:20], dtype=np.uint8)
    x = np.asarray(x, dtype=np.uint8)
    return t0[x & 7] ^ t1[(x >> 3) & 7] ^ t2[x >> 6]


# ---- GF(2^16) as four byte maps (what the gfx950 w = 16 kernel applies) --------------------------
def perm_quads16(coeff: np.ndarray) -> np.ndarray:
    """(m, k) GF(2^16) coefficients -> (m, k, 4, 8) uint32 v_perm records, the four byte maps of
    each multiply in the order q = 2 * src_byte + dst_byte (``csrc/include/gfrs/gf65536.h``
    perm_quad): c * (l | h << 8) = [L_ll(l) ^ L_hl(h)] | [L_lh(l) ^ L_hh(h)] << 8. Vectorised over
    all coefficients."""
    f = field(16)
    c = np.asarray(coeff, dtype=np.int64)
    m, k = c.shape
    imgs = f.mul(c.reshape(-1, 1), (1 << np.arange(16)).reshape(1, -1))  # (m*k, 16) images of the bits
    out = np.zeros((m * k, 4, 8), dtype=np.uint32)

    def table(basis: np.ndarray, nbits: int) -> np.ndarray:  # (N, nbits) -> (N, 2**nbits) XOR combos
        t = np.zeros((basis.shape[0], 1 << nbits), dtype=np.int64)
        for v in range(1, 1 << nbits):
            for b in range(nbits):
                if v >> b & 1:
                    t[:, v] ^= basis[:, b]
        return t

    def pack(t: np.ndarray) -> np.ndarray:  # (N, 4) bytes -> (N,) little-endian words
        return (t[:, 0] | (t[:, 1] << 8) | (t[:, 2] << 16) | (t[:, 3] << 24)).astype(np.uint32)

    for src in range(2):
        for dst in range(2):
            basis = (imgs[:, 8 * src: 8 * src + 8] >> (8 * dst)) & 0xFF  # (N, 8) byte images
            t0, t1, t2 = table(basis[:, 0:3], 3), table(basis[:, 3:6], 3), table(basis[:, 6:8], 2)
            q = 2 * src + dst
            out[:, q, 0], out[:, q, 1] = pack(t0[:, 0:4]), pack(t0[:, 4:8])
            out[:, q, 2], out[:, q, 3] = pack(t1[:, 0:4]), pack(t1[:, 4:8])
            out[:, q, 4] = pack(t2)
    return out.reshape(m, k, 4, 8)


def quad_apply16(quad: np.ndarray, x: np.ndarray) -> np.ndarray:
    """Host emulation of the device lookup of one GF(2^16) coefficient on uint16 symbols (tests)."""
    x = np.asarray(x, dtype=np.uint16)
    lo, hi = (x & 0xFF).astype(np.uint8), (x >> 8).astype(np.uint8)
    ol = perm_apply(quad[0], lo) ^ perm_apply(quad[2], hi)
    oh = perm_apply(quad[1], lo) ^ perm_apply(quad[3], hi)
    return (ol.astype(np.uint16) | (oh.astype(np.uint16) << 8)).astype(np.uint16)
