"""The xGMI-sharded k_batch decodes the winner's global node index from its packed key
(kgpu_kernels.hip rank40_inv): the tie-break hash rank40 must be a bijection on 40 bits and
rank40_inv its inverse, for both tie-break modes.  Host restatement of the two device functions
(constants as in the kernel), checked on random and edge indices."""
import random

from oracle.refsched import tiebreak

M = (1 << 40) - 1


def rank40_inv(k, x, mode):
    if mode == 1:
        return M - x
    x ^= (k >> 24) & M
    x ^= x >> 23
    x = (x * 0x38E12D471B) & M
    x ^= (x >> 19) ^ (x >> 38)
    x = (x * 0xB38E39396D) & M
    x ^= k & M
    return x


def test_rank40_inverse_round_trip():
    r = random.Random(7)
    for mode in (tiebreak.MODE_HASH, tiebreak.MODE_FIRST):
        for seq in range(40):
            k = tiebreak.pod_key(0x7B, seq)
            idx = [0, 1, 2, 999_999, (1 << 20) - 1, (1 << 40) - 1] + [r.randrange(1 << 40) for _ in range(200)]
            for i in idx:
                x = (M - i) if mode == tiebreak.MODE_FIRST else tiebreak.rank40(k, i)
                assert rank40_inv(k, x, mode) == i, (mode, seq, i)


def test_tiebreak_keys_np_matches_scalar_keys():
    """kgpu.tiebreak.keys_np (the extender's vectorized selectHost over candidates) equals key() per node."""
    import random

    import numpy as np
    from kgpu import tiebreak as T
    rng = random.Random(7)
    for mode in (T.MODE_HASH, T.MODE_FIRST):
        for _ in range(100):
            seed, seq = rng.getrandbits(64), rng.getrandbits(24)
            idx = np.array([rng.randrange(1 << 21) for _ in range(40)])
            sc = np.array([rng.randrange(1 << 23) for _ in range(40)])
            got = [int(x) for x in T.keys_np(sc, idx, seed, seq, mode)]
            assert got == [T.key(int(s), int(i), seed, seq, mode) for s, i in zip(sc, idx)]
