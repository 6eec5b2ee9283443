"""Test infrastructure only: tests/ import this file; the product never does.

Host restatement of the engine's DEVICE minibatch sampler (sampling = 'device', the
non-parity throughput mode of SURVEY.md section 7, hard part 1), following
distributed-optimization_amd/csrc/kernels.hip: `philox4x32` and `floyd_sample`:

* Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as
  1, 2, 3", SC'11): multipliers 0xD2511F53 / 0xCD9E8D57, key bumps 0x9E3779B9 /
  0xBB67AE85, ten rounds.
* Draw k of worker w in round t: word k % 4 of philox(counter = (k // 4, w, t mod 2^32,
  t >> 32), key = (seed mod 2^32, seed >> 32)), mapped to [0, j] as (u * (j + 1)) >> 32.
* Floyd's algorithm: for j = m - nb .. m - 1, t = draw in [0, j]; take t unless already
  taken, else take j -- a uniform nb-subset of [0, m), nb = min(b, m).

This is not the reference's algorithm (the reference draws np.random.choice from the
legacy MT19937 stream, restated bit-exactly in csrc/sampler.cpp); it pins the device
sampler's output so the GPU tests can replay the same minibatches through the index path.
"""
import numpy as np

_M0, _M1, _W0, _W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
_U32 = 0xFFFFFFFF


def philox4x32(ctr, k0, k1):
    x, y, z, w = ctr
    for _ in range(10):
        p0, p1 = _M0 * x, _M1 * z
        x, y, z, w = ((p1 >> 32) ^ y ^ k0) & _U32, p1 & _U32, ((p0 >> 32) ^ w ^ k1) & _U32, p0 & _U32
        k0, k1 = (k0 + _W0) & _U32, (k1 + _W1) & _U32
    return x, y, z, w


def minibatch(seed, rnd, worker, m, b):
    """Sorted row ids of worker `worker`'s minibatch in round `rnd` (global ids)."""
    nb = min(b, m)
    taken = np.zeros(max(m, 1), dtype=bool)
    r = None
    for k, j in enumerate(range(m - nb, m)):
        if k % 4 == 0:
            r = philox4x32((k >> 2, worker & _U32, rnd & _U32, (rnd >> 32) & _U32), seed & _U32, (seed >> 32) & _U32)
        t = (r[k % 4] * (j + 1)) >> 32
        if taken[t]:
            taken[j] = True
        else:
            taken[t] = True
    return np.flatnonzero(taken[:m])


def rounds(seed, t0, T, shard_rows, b, first_worker=0):
    """[T, N, b] int32 indices (ascending per worker, -1 padded) of rounds t0 .. t0+T-1,
    in the layout of dopt_mt_choice_rounds."""
    out = np.full((T, len(shard_rows), b), -1, dtype=np.int32)
    for h in range(T):
        for i, m in enumerate(shard_rows):
            sel = minibatch(seed, t0 + h, first_worker + i, int(m), b)
            out[h, i, :len(sel)] = sel
    return out
