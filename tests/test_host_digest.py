"""The drop-in trainers' engine cache key (trainer._fingerprint over dopt_host_digest): every byte of
the host shards is hashed on every run by default, so an in-place edit anywhere reloads the shards
(the round-4 sampled key missed edits between its 64 sampled pieces); the sampled key is an
explicit opt-in (config content_key='sampled').  Host code only: no GPU needed."""
import numpy as np
import pytest

import _dopt
import trainer


def test_digest_sees_every_byte_order_and_length():
    rng = np.random.default_rng(0)
    a = rng.standard_normal((4 << 20) // 8 + 5)  # 4 MiB chunks + a ragged tail chunk
    b = rng.integers(0, 9, 1001).astype(np.int64)
    d0 = _dopt.host_digest([a, b])
    assert len(d0) == 32 and d0 == _dopt.host_digest([a.copy(), b.copy()])
    assert all(_dopt.host_digest([a, b], threads=k) == d0 for k in (1, 2, 7))
    for pos in (0, 1, (4 << 20) // 8 - 1, (4 << 20) // 8, a.size - 1):
        e = a.copy()
        e[pos] = np.nextafter(e[pos], np.inf)  # one bit of one element
        assert _dopt.host_digest([e, b]) != d0, pos
    assert _dopt.host_digest([b, a]) != d0
    assert _dopt.host_digest([a[:-1], b]) != d0
    assert _dopt.host_digest([a, b[:-1]]) != d0
    assert _dopt.host_digest([]) != _dopt.host_digest([np.zeros(0)])


def test_fingerprint_sees_in_place_edits_of_large_shards():
    X = np.zeros(((70 << 20) // 8 // 64 + 3, 64))  # > 64 MiB: the size the round-4 key sampled
    y = np.ones(X.shape[0])
    k0 = trainer._fingerprint([X, y])
    row = X.shape[0] // 64 + 17  # between two of the sampled key's 256-byte pieces
    X[row, 5] = 1.0
    k1 = trainer._fingerprint([X, y])
    assert k1 != k0
    y[3] = -1.0
    assert trainer._fingerprint([X, y]) not in (k0, k1)
    assert trainer._fingerprint([X.astype(np.float32), y]) != trainer._fingerprint([X, y])


def test_sampled_key_is_opt_in_and_documented():
    X = np.zeros(((70 << 20) // 8 // 64 + 3, 64))
    y = np.ones(X.shape[0])
    trainer.forget_data()
    s0 = trainer._fingerprint([X, y], sampled=True)
    assert s0 == trainer._fingerprint([X, y])  # the same digest as the full key on first sight
    X[X.shape[0] // 64 + 17, 5] = 1.0
    assert trainer._fingerprint([X, y], sampled=True) == s0  # the edit the sample misses
    trainer.forget_data()
    assert trainer._fingerprint([X, y], sampled=True) != s0
    assert trainer._sampled_key({}) is False and trainer._sampled_key({"content_key": "sampled"}) is True
    with pytest.raises(ValueError):
        trainer._sampled_key({"content_key": "ids"})
