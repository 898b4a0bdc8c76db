"""Test infrastructure: a numpy restatement of Philox4x32-10 (Salmon et al., SC'11; the Random123 constants and
round structure) and of cn_uniform_philox's mapping to [0, 1), the checker of the device generator."""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """ctr: uint32 [..., 4], key: uint32 [2] -> uint32 [..., 4]."""
    c = [ctr[..., i].astype(np.uint64) for i in range(4)]
    k0, k1 = np.uint32(key[0]), np.uint32(key[1])
    with np.errstate(over="ignore"):
        for r in range(10):
            if r:
                k0 = np.uint32(k0 + W0)
                k1 = np.uint32(k1 + W1)
            p0 = M0 * c[0]
            p1 = M1 * c[2]
            n0 = (p1 >> np.uint64(32)) ^ c[1] ^ np.uint64(k0)
            n2 = (p0 >> np.uint64(32)) ^ c[3] ^ np.uint64(k1)
            c = [n0 & MASK, p1 & MASK, n2 & MASK, p0 & MASK]
    return np.stack([x.astype(np.uint32) for x in c], -1)


def uniform(n, seed, offset):
    """cn_uniform_philox's out[0 .. n) for (seed, offset)."""
    g = np.arange((n + 3) // 4, dtype=np.uint64)
    ctr = np.stack([g & MASK, g >> np.uint64(32), np.full_like(g, offset & 0xFFFFFFFF),
                    np.full_like(g, offset >> 32)], -1).astype(np.uint32)
    words = philox4x32_10(ctr, (seed & 0xFFFFFFFF, seed >> 32)).reshape(-1)[:n]
    return (words >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
