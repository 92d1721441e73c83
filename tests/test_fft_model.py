"""CPU checks of the additive-FFT codec's math (tests/fft_model.py mirrors
rs_fft.hip's transform structure: LCH novel basis over the subspace of
integer-labelled field elements, twiddles W_j(lambda), recursive systematic
solve, pruned output FFT).  Pins that the structure the kernel unrolls is
bit-identical to klauspost v1.9.1's encode matrix for every geometry the
build specialises and for odd ones, and that the multiply count matches the
design figure (462 constant multiplies at N=128, k=44)."""
import numpy as np
import pytest

import fft_model as fm
import rbc_oracle as orc


@pytest.mark.parametrize("n,f", [(4, 1), (16, 5), (64, 21), (128, 42), (256, 85), (7, 2), (13, 4), (100, 20),
                                 (128, 10), (2, 0), (33, 8), (256, 0)])
def test_fft_encode_equals_klauspost_matrix(n, f):
    k = n - 2 * f
    rng = np.random.default_rng(n * 31 + f)
    data = [rng.integers(0, 256, 37, dtype=np.uint8) for _ in range(k)]
    want = orc.gf_rows(orc.encode_matrix(k, n)[k:], data)
    got = fm.encode(k, n, data)
    assert all(np.array_equal(g, d) for g, d in zip(got[:k], data))
    assert all(np.array_equal(g, w) for g, w in zip(got[k:], want))


def test_fft_roundtrip_and_twiddles():
    # FFT o IFFT = id on every coset size used by the kernels
    rng = np.random.default_rng(5)
    for m in range(1, 8):
        for lam in (0, 1 << m, 3 << m) if m < 7 else (0, 128):
            v = [rng.integers(0, 256, 8, dtype=np.uint8) for _ in range(1 << m)]
            back = fm.fft(m, lam, fm.ifft(m, lam, list(v)))
            assert all(np.array_equal(a, b) for a, b in zip(back, v))
    # W_j vanishes on V_j and is 1 at 2^j (normalised subspace polynomial)
    for j in range(8):
        assert all(fm.WN[j][x] == 0 for x in range(1 << j))
        assert fm.WN[j][1 << j] == 1


def test_fft_multiply_count_matches_design():
    cnt = fm.Counter()
    data = [np.zeros(1, np.uint8) for _ in range(44)]
    fm.encode(44, 128, data, cnt)
    assert cnt.mul == 462  # vs 84 * 44 = 3696 matrix MACs
