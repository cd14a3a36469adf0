"""Host mirror of the pair-hash dropout bits (csrc/common.h ``pair_hash``).

The post-LN sublayers draw their branch dropout inside the producing GEMM's epilogue
(csrc/gemm256.hip EPI 7) and the LayerNorm backward regenerates the same bits
(csrc/norm.hip ``dropout_keep_pair``).  This module computes that mask on the host so the
tests can build an exact torch reference; uint64 numpy arithmetic wraps modulo 2^64, which
keeps every low-32-bit product exact."""
import numpy as np
import torch

_M32 = np.uint64(0xFFFFFFFF)


def _u(x):
    return np.asarray(x, dtype=np.uint64) & _M32


def lowbias32(x):
    x = _u(x)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & _M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & _M32
    x ^= x >> np.uint64(16)
    return x


def mix32(x):
    x = _u(x)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & _M32
    x ^= x >> np.uint64(15)
    return x


def pair_seedmix(seed, offset):
    return lowbias32(_u(seed) ^ lowbias32(((_u(offset) * np.uint64(0xC2B2AE3D)) & _M32) ^ np.uint64(0x68E31DA4)))


def pair_thr16(p):
    return int(np.float32(p) * np.float32(65536.0) + np.float32(0.5))


def pair_keep_mask(seed, offset, R, D, p):
    """[R, D] bool: element (row, col) of a [R, D] branch output is kept."""
    sm = pair_seedmix(seed, offset)
    rows = np.arange(R, dtype=np.uint64)[:, None]
    cols = np.arange(D, dtype=np.uint64)[None, :]
    h = mix32(sm ^ ((rows * np.uint64(0x9E3779B1)) & _M32) ^ (((cols >> np.uint64(1)) * np.uint64(0x85EBCA77)) & _M32))
    half = np.where((cols & np.uint64(1)) == np.uint64(1), h >> np.uint64(16), h & np.uint64(0xFFFF))
    return torch.from_numpy(half >= np.uint64(pair_thr16(p)))
