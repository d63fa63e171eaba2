"""Deterministic synthetic stake networks.

stake(i)  = floor(1.5e16 / (i + 1)) + (philox_u64(0x5EED0001, i) mod 1e9), floored at 1 SOL
pubkey(i) = 32 bytes of Philox(0x5EED0002, i) blocks 0 and 1 (little-endian words)
Nodes are then re-indexed by the rank of their base58 pubkey string (node id).
The generator is vectorised Philox4x32-10 in numpy (the same counter layout as
the engine's streams: key = seed halves, counter = {block, a, b, purpose}).
"""
import numpy as np

SEED_STAKE = 0x5EED0001
SEED_PUBKEY = 0x5EED0002
M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, seed):
    """Vectorised Philox4x32-10 over uint32 arrays; returns four uint32 arrays."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint64) for x in (c0, c1, c2, c3))
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + W0) & 0xFFFFFFFF
            k1 = (k1 + W1) & 0xFFFFFFFF
        p0 = M0 * c0
        p1 = M1 * c2
        n0 = (p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0)
        n2 = (p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1)
        c0, c1, c2, c3 = n0, p1 & MASK32, n2, p0 & MASK32
    return c0, c1, c2, c3


def philox_u64(seed, idx, purpose=0, b=0, block=0, which=0):
    idx = np.asarray(idx, dtype=np.uint64)
    z = np.zeros_like(idx)
    o0, o1, o2, o3 = philox4x32_10(z + np.uint64(block), idx, z + np.uint64(b), z + np.uint64(purpose), seed)
    if which == 0:
        return o0 | (o1 << np.uint64(32))
    return o2 | (o3 << np.uint64(32))


def power_law_stakes(n):
    i = np.arange(n, dtype=np.uint64)
    base = np.uint64(15_000_000_000_000_000) // (i + np.uint64(1))
    jitter = philox_u64(SEED_STAKE, i) % np.uint64(1_000_000_000)
    return np.maximum(base + jitter, np.uint64(1_000_000_000))


def pubkeys(n):
    i = np.arange(n, dtype=np.uint64)
    words = []
    for block in (0, 1):
        z = np.zeros_like(i)
        o = philox4x32_10(z + np.uint64(block), i, z, z, SEED_PUBKEY)
        words.extend(o)
    w = np.stack(words, axis=1).astype("<u4")  # n x 8 little-endian words
    return [bytes(row.tobytes()) for row in w]


def network(n):
    """(pubkeys in id order, stakes in id order) for the synthetic power-law network."""
    from . import b58encode
    pks = pubkeys(n)
    st = power_law_stakes(n)
    strs = [b58encode(p) for p in pks]
    if len(set(strs)) != n:
        raise ValueError("pubkey collision")
    order = sorted(range(n), key=lambda k: strs[k])
    return [pks[k] for k in order], np.ascontiguousarray(st[order])
