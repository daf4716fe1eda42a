"""Test helpers: deterministic data identical to oracle/gen_golden.c."""
import hashlib

import numpy as np

GOLDEN = 0x9E3779B97F4A7C15
MASK = (1 << 64) - 1


def case_seed(n: int, k: int, cs: int) -> int:
    """seed = 1000003*n + 10007*k + cs (gen_golden.c case_seed)."""
    return 1000003 * n + 10007 * k + cs


def fill_bytes(nbytes: int, seed: int) -> np.ndarray:
    """splitmix64 little-endian byte stream (orc_fill_bytes / nxec_fill_random), vectorised."""
    words = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        i = np.arange(1, words + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:nbytes].copy()


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def hexbytes(s: str) -> np.ndarray:
    return np.frombuffer(bytes.fromhex(s), dtype=np.uint8)


def mixed_pattern(n: int, k: int, e: int):
    """gen_golden.c mixed_pattern."""
    nd, np_ = e // 2, e - e // 2
    dsel = [1, 4, 7, 10, 13]
    return [dsel[i] % k for i in range(nd)] + [n - 3, n - 1][2 - np_:]


def checksum64(a: np.ndarray) -> int:
    """nxec_checksum: sum_i word_i * (2i+1) mod 2^64 over LE 8-byte words (zero-padded tail)."""
    b = np.ascontiguousarray(a, dtype=np.uint8)
    pad = (-len(b)) % 8
    if pad:
        b = np.concatenate([b, np.zeros(pad, dtype=np.uint8)])
    w = b.view("<u8")
    with np.errstate(over="ignore"):
        m = np.arange(len(w), dtype=np.uint64) * np.uint64(2) + np.uint64(1)
        return int(np.sum(w * m, dtype=np.uint64))
