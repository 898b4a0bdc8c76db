"""The numpy Philox4x32-10 (tests/philox_ref.py, the checker of cn_uniform_philox) against the Random123
known-answer vectors (kat_vectors: philox4x32 10 rounds)."""
import numpy as np

from philox_ref import philox4x32_10, uniform

KAT = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
       ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
       ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
        (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]


def test_philox_known_answers():
    for ctr, key, want in KAT:
        got = philox4x32_10(np.array([ctr], dtype=np.uint32), key)[0]
        assert [int(x) for x in got] == list(want), [hex(int(x)) for x in got]


def test_uniform_mapping():
    u = uniform(10007, seed=0x1234567890ABCDEF, offset=(5 << 32) + 7)
    assert u.dtype == np.float32 and u.shape == (10007,)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(float(u.mean()) - 0.5) < 0.01
    # word i % 4 of group i // 4: the first group is the generator's first block
    blk = philox4x32_10(np.array([[0, 0, 7, 5]], dtype=np.uint32), (0x90ABCDEF, 0x12345678))[0]
    assert np.array_equal(u[:4], (blk >> 8).astype(np.float32) / np.float32(16777216.0))
