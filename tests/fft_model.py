#!/usr/bin/env python3
"""Python model of the additive-FFT Reed-Solomon encoder used by the gfx950
`rs_fft_kernel` (test infrastructure: pins the transform's math against the
oracle on the CPU; not product code).

klauspost/reedsolomon v1.9.1's code (oracle/rbc_oracle.py build_matrix) is
M = V * inv(V[:k]), V[r][c] = r^c over GF(2^8)/0x11D: shard r of the codeword
is P(r) for the unique P with deg P < k and P(j) = data_j (j < k), the points
being the field elements with integer labels 0..N-1.  Those labels are the
GF(2)-subspace V_n = span{1, 2, 4, ..., 2^(n-1)}, so P can be moved between
evaluations and coefficients in the Lin-Chung-Han novel polynomial basis
X_i = prod_{j in bits(i)} W_j, W_j = s_j / s_j(2^j), s_j the vanishing
polynomial of V_j, with O(W log W) butterflies.  deg P < k  <=>  the novel
coefficients c_i vanish for i >= k, so the systematic encode is:
  coeffs = solve(n, 0, data, k)        (recursive, only power-of-two IFFTs)
  shards[k..N) = FFT(coeffs) restricted to the needed outputs.
Every output byte equals the matrix product bit-for-bit (same linear map).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import rbc_oracle as orc  # noqa: E402  (tests/ may use the oracle as the checker)

MUL = orc.MUL


def gmul(a, b):
    return int(MUL[a, b])


def ginv(a):
    return orc.gal_div(1, a)


# s_j(x) for all x (linearized): s_0 = x, s_{j+1}(x) = s_j(x) * (s_j(x) + s_j(2^j))
S = [list(range(256))]
for _j in range(8):
    prev = S[-1]
    sv = prev[1 << _j]
    S.append([gmul(prev[x], prev[x] ^ sv) for x in range(256)])
WN = [[gmul(S[j][x], ginv(S[j][1 << j])) if S[j][1 << j] else 0 for x in range(256)] for j in range(8)]


def twiddle(j, lam):
    """W_j(lambda): the butterfly constant of layer j on coset lambda."""
    return WN[j][lam]


class Counter:
    def __init__(self):
        self.mul = 0     # general multiplies (omega not in {0,1})
        self.xor = 0


def fft(m, lam, c, cnt=None, need=None):
    """Evaluations of sum c_i X_i on lam + {0..2^m}.  c: list of rows (None = known zero)."""
    if m == 0:
        return [c[0]]
    h = 1 << (m - 1)
    w = twiddle(m - 1, lam)
    a, b = c[:h], c[h:]
    a2, b2 = [], []
    for x, y in zip(a, b):
        if y is None:
            a2.append(x)
            b2.append(x)
            continue
        if w == 0:
            t = x
        else:
            t = MUL[w, y] if w != 1 else y
            if cnt is not None and w != 1:
                cnt.mul += 1
            if x is not None:
                t = t ^ x
                if cnt is not None:
                    cnt.xor += 1
        a2.append(t)
        b2.append(y if t is None else t ^ y)
        if cnt is not None and t is not None:
            cnt.xor += 1
    return fft(m - 1, lam, a2, cnt) + fft(m - 1, lam + h, b2, cnt)


def ifft(m, lam, v, cnt=None):
    if m == 0:
        return [v[0]]
    h = 1 << (m - 1)
    w = twiddle(m - 1, lam)
    a2 = ifft(m - 1, lam, v[:h], cnt)
    b2 = ifft(m - 1, lam + h, v[h:], cnt)
    a, b = [], []
    for x, y in zip(a2, b2):
        bb = x ^ y
        aa = x ^ MUL[w, bb] if w else x
        if cnt is not None:
            cnt.xor += 1 + (1 if w else 0)
            cnt.mul += 1 if w not in (0, 1) else 0
        a.append(aa)
        b.append(bb)
    return a + b


def solve(m, lam, vals, t, cnt=None):
    """Novel-basis coefficients (2^m rows, None beyond t) of the polynomial with
    support [0, t) whose evaluations on the first t points of lam+V_m are vals."""
    size = 1 << m
    if t == size:
        return ifft(m, lam, list(vals), cnt)
    h = size >> 1
    if t <= h:
        return solve(m - 1, lam, vals, t, cnt) + [None] * h
    w = twiddle(m - 1, lam)
    g = ifft(m - 1, lam, list(vals[:h]), cnt)           # P0 + w P1
    hv = fft(m - 1, lam + h, g, cnt)                    # FFT(g) on the upper coset
    tp = t - h
    d = [vals[h + i] ^ hv[i] for i in range(tp)]        # FFT(P1) on its first tp points
    if cnt is not None:
        cnt.xor += tp
    p1 = solve(m - 1, lam + h, d, tp, cnt)
    p0 = []
    for x, y in zip(g, p1):
        if y is None or w == 0:
            p0.append(x)
        else:
            p0.append(x ^ (MUL[w, y] if w != 1 else y))
            if cnt is not None:
                cnt.xor += 1
                cnt.mul += 1 if w != 1 else 0
    return p0 + p1


def encode(k, n_total, data, cnt=None):
    """data: k rows (uint8 arrays) -> n_total rows (systematic codeword)."""
    m = max(1, (n_total - 1).bit_length())
    coef = solve(m, 0, data, k, cnt)
    ev = fft(m, 0, coef, cnt)
    return ev[:n_total]


def main():
    rng = np.random.default_rng(1)
    for (n, f) in [(4, 1), (16, 5), (64, 21), (128, 42), (256, 85), (7, 2), (13, 4), (100, 20), (128, 10)]:
        k = n - 2 * f
        data = [rng.integers(0, 256, 24, dtype=np.uint8) for _ in range(k)]
        want = orc.gf_rows(orc.encode_matrix(k, n)[k:], data)
        cnt = Counter()
        got = encode(k, n, data, cnt)
        ok = all(np.array_equal(g, w) for g, w in zip(got[k:], want)) and all(
            np.array_equal(g, d) for g, d in zip(got[:k], data))
        print(f"N={n:3d} k={k:3d}: {'OK ' if ok else 'BAD'} muls={cnt.mul} xors={cnt.xor} "
              f"(matrix MACs {k * (n - k)})")


if __name__ == "__main__":
    main()
