"""The build's selectHost tie-break on the host side (DESIGN.md 'Determinism contract'): the same
packed key the kernels form (kgpu_kernels.hip pod_tie_key / rank40), for host code that ranks a
subset of the device's nodes -- the extender's candidate list (kgpu/extender.py).

    key = score << 40 | rank40(splitmix64(seed ^ seq * phi), node_index)

The reference breaks equal top scores by reservoir sampling over math/rand
(core/generic_scheduler.go:217-238); the build fixes a deterministic rule instead."""
MASK40 = (1 << 40) - 1
M64 = (1 << 64) - 1
MODE_HASH, MODE_FIRST = 0, 1
_PHI = 0x9E3779B97F4A7C15


def _splitmix64(x):
    x = (x + _PHI) & M64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def rank(seed, seq, idx, mode=MODE_HASH):
    """Low 40 bits of the key of node `idx` (global Snapshot.List() index) for pod sequence `seq`."""
    if mode == MODE_FIRST:
        return MASK40 - idx
    k = _splitmix64((seed ^ ((seq * _PHI) & M64)) & M64)
    x = (idx & MASK40) ^ (k & MASK40)
    x = (x * 0xD6E8FEB865) & MASK40
    x ^= x >> 19
    x = (x * 0x94D049BB13) & MASK40
    x ^= x >> 23
    return x ^ ((k >> 24) & MASK40)


def key(score, idx, seed, seq, mode=MODE_HASH):
    return (score << 40) | rank(seed, seq, idx, mode)


def keys_np(scores, idx, seed, seq, mode=MODE_HASH):
    """key() over arrays of scores and node indices (numpy uint64; the 40-bit products wrap mod 2^64,
    which keeps their low 40 bits exact)."""
    import numpy as np
    idx = np.asarray(idx, np.uint64)
    if mode == MODE_FIRST:
        r = np.uint64(MASK40) - idx
    else:
        k = _splitmix64((seed ^ ((seq * _PHI) & M64)) & M64)
        m = np.uint64(MASK40)
        with np.errstate(over="ignore"):
            x = (idx & m) ^ np.uint64(k & MASK40)
            x = (x * np.uint64(0xD6E8FEB865)) & m
            x ^= x >> np.uint64(19)
            x = (x * np.uint64(0x94D049BB13)) & m
            x ^= x >> np.uint64(23)
        r = x ^ np.uint64((k >> 24) & MASK40)
    return (np.asarray(scores, np.uint64) << np.uint64(40)) | r
