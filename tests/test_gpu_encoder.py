"""reedsolomon.Encoder mirror on the GPU (rbc_rs_*, klauspost v1.9.1 held at
rbc/rbc.go:20): Update against the oracle's restatement of
reedsolomon.go Update / updateParityShards, including Go's argument checks
and its side effect on the old data shards."""
import numpy as np
import pytest

import rbc_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,p,S,nchg", [(5, 5, 2, 1), (44, 84, 1001, 7), (44, 84, 23832, 44), (86, 170, 763, 3),
                                        (1, 3, 64, 1), (17, 4, 4097, 5)])
def test_update_matches_oracle(gpu, k, p, S, nchg):
    ca = gpu
    rng = np.random.default_rng(k * 1000 + S)
    enc = ca.Encoder(k, p)
    ref = orc.Encoder(k, p)
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
    shards = [d.copy() for d in data] + [np.zeros(S, np.uint8) for _ in range(p)]
    ref.encode(shards)
    new = [None] * k
    for c in rng.choice(k, size=nchg, replace=False):
        new[c] = rng.integers(0, 256, S, dtype=np.uint8)
    got = [s.copy() for s in shards]
    want = [s.copy() for s in shards]
    enc.update(got, new)
    ref.update(want, new)
    for i in range(k + p):
        assert np.array_equal(got[i], want[i]), i
    # the updated parity is the encoding of the new data
    full = [(new[c] if new[c] is not None else data[c]) for c in range(k)] + [np.zeros(S, np.uint8)] * p
    ref.encode(full)
    for r in range(p):
        assert np.array_equal(got[k + r], full[k + r]), r
    assert enc.verify(full)


def test_update_argument_checks_follow_go_order(gpu):
    ca = gpu
    enc = ca.Encoder(3, 2)
    S = 8
    sh = [np.ones(S, np.uint8) for _ in range(5)]
    new = [np.zeros(S, np.uint8), None, None]
    cases = [
        (sh[:4], new, -3),                                                    # ErrTooFewShards
        (sh, new[:2], -3),
        (sh + [np.ones(S, np.uint8)], new, -3),                               # len(shards) != Shards
        (sh, new + [None], -3),                                               # len(new) != DataShards
        (sh, [None, None, None], -4),                                         # ErrShardNoData
        ([np.ones(S, np.uint8)] * 4 + [np.ones(S + 1, np.uint8)], new, -5),   # ErrShardSize (shards)
        ([None] + sh[1:], new, -13),                                          # ErrInvalidInput
        (sh[:4] + [None], new, -13),
        (sh, [np.zeros(S + 2, np.uint8), None, None], -5),                    # new shard of another size
    ]
    for shards, nd, code in cases:
        with pytest.raises(ca.RBCError) as e:
            enc.update([None if s is None else s.copy() for s in shards], nd)
        assert e.value.code == code, (len(shards), code)
