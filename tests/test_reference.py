"""CPU tests of the host oracles used to check the HIP kernels."""
import hashlib

import numpy as np

from tritonk8ssupervisor_amd.ops import reference as ref


def test_philox_known_answers():
    # Random123 kat_vectors for philox4x32_10.
    cases = [
        ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
        ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
        ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
         (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
    ]
    for ctr, key, want in cases:
        got = ref.philox4x32_10(np.array([ctr], dtype=np.uint32), key)[0]
        assert tuple(int(x) for x in got) == want


def test_philox_bytes_layout():
    b = ref.philox_bytes(64, seed=0)
    assert len(b) == 64
    words = np.frombuffer(b, dtype="<u4")
    assert tuple(int(x) for x in words[:4]) == (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)
    # different seeds give different streams
    assert ref.philox_bytes(64, seed=1) != b


def test_md5_tree_small_is_plain_md5():
    for n in (0, 1, 55, 56, 63, 64, 1000, 1024):
        data = bytes(range(256)) * (n // 256 + 1)
        data = data[:n]
        assert ref.md5_tree(data, 1024) == hashlib.md5(data).digest()


def test_md5_tree_levels():
    md5 = lambda b: hashlib.md5(b).digest()
    # 5 leaves (the last partial): a parent of four and a parent of one, then the root
    data = ref.philox_bytes(4096 + 512, seed=7)
    d = [md5(data[i : i + 1024]) for i in range(0, len(data), 1024)]
    assert ref.md5_tree(data, 1024) == md5(md5(b"".join(d[:4])) + md5(d[4]))
    # 128 leaves: 32 -> 8 -> 2 -> 1
    big = ref.philox_bytes(1 << 17, seed=3)
    level = [md5(big[i : i + 1024]) for i in range(0, len(big), 1024)]
    for want in (32, 8, 2, 1):
        level = [md5(b"".join(level[i : i + 4])) for i in range(0, len(level), 4)]
        assert len(level) == want
    assert ref.md5_tree(big, 1024) == level[0]
    # two chunks: the root hashes the two leaf digests (32 bytes)
    two = data[:2048]
    assert ref.md5_tree(two, 1024) == md5(md5(two[:1024]) + md5(two[1024:]))


def test_allreduce_expected():
    e = ref.allreduce_expected(10, 4)
    i = np.arange(10)
    assert np.array_equal(e, (10 + 4 * (i % 7)).astype(np.float32))
