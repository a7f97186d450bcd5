"""ORACLE (test infrastructure only) -- the build's deterministic selectHost tie-break.

The reference breaks equal top scores by reservoir sampling with the global math/rand
source (pkg/scheduler/core/generic_scheduler.go:217-238), which is not reproducible.  The
build replaces it by a packed 64-bit key, identical on CPU and GPU (DESIGN.md 'Determinism
contract'):

    key = score << 40 | rank40(seed, pod_seq, node_index)

rank40 is a bijection of the 40-bit node index (xor / odd multiply / xorshift steps, each
invertible mod 2^40), so the argmax is unique; every tied node is equally likely to win
across pods, like the reference's reservoir sampling.  MODE_FIRST ranks by snapshot order
(first maximum wins).  Scores must be < 2^23.
"""
MASK40 = (1 << 40) - 1
M64 = (1 << 64) - 1
MODE_HASH, MODE_FIRST = 0, 1
C1 = 0x9E3779B97F4A7C15
C_MUL1 = 0xD6E8FEB865 | 1   # odd, < 2^40
C_MUL2 = 0x94D049BB13 | 1


def splitmix64(x):
    x = (x + C1) & M64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def pod_key(seed, pod_seq):
    return splitmix64((seed ^ ((pod_seq * C1) & M64)) & M64)


def rank40(k, idx):
    x = idx & MASK40
    x ^= k & MASK40
    x = (x * C_MUL1) & MASK40
    x ^= x >> 19
    x = (x * C_MUL2) & MASK40
    x ^= x >> 23
    x ^= (k >> 24) & MASK40
    return x


def key(score, idx, pod_seq, seed, mode=MODE_HASH):
    if mode == MODE_FIRST:
        r = MASK40 - idx
    else:
        r = rank40(pod_key(seed, pod_seq), idx)
    return (score << 40) | r
